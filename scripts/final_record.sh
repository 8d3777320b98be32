#!/bin/bash
# The round's record of the benched tree in ONE session: PMC passes of the fp16 cfg2 quick bench
# (FETCH_SIZE / WRITE_SIZE / MFMA in separate runs) -> <rec>/pmc_traffic.json, copied into profiles/<rec>/ on the box
# first so that the default bench line that follows cites it as traffic_source; then the default bench (headline +
# modes + cfg3 + cfg4 + CPU baseline) and a rocprofv3 kernel-trace/stats pass of the fp16 cfg2 quick bench (one mode,
# one workload) with its per-level breakdown.  Everything lands in gpurun_out/<rec>/.   REC=r03_final bash scripts/final_record.sh
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
REC=${REC:-r03_final}
O=gpurun_out/$REC
mkdir -p $O profiles/$REC
echo "cpus: os.cpu_count=$(python -c 'import os;print(os.cpu_count())') affinity=$(python -c 'import os;print(len(os.sched_getaffinity(0)))') nproc=$(nproc)" > $O/host.txt
grep -m1 "model name" /proc/cpuinfo >> $O/host.txt
git_rev=$(cat .git_rev 2>/dev/null || echo unknown); echo "tree: $git_rev" >> $O/host.txt
SUFFIX=_$REC bash scripts/pmc_pass.sh > $O/pmc_pass.log 2>&1
for p in fetch write mfma; do cp gpurun_out/pmc_${p}_$REC/run_kernel_stats.csv $O/pmc_${p}_kernel_stats.csv; done
python scripts/pmc_traffic.py gpurun_out/pmc_fetch_$REC gpurun_out/pmc_write_$REC gpurun_out/pmc_mfma_$REC $O/pmc_traffic.json
cp $O/pmc_traffic.json profiles/$REC/pmc_traffic.json
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench_stderr.txt
tail -c 400 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$REC -o run --output-format csv -- \
    python bench.py --steps 10 --warmup 3 --quick > $O/prof_bench.json 2> $O/prof_bench_stderr.txt
cp gpurun_out/prof_$REC/run_kernel_stats.csv $O/kernel_stats.csv
python scripts/trace_levels.py gpurun_out/prof_$REC/run_kernel_trace.csv > $O/trace_levels.txt
rm -rf gpurun_out/prof_$REC gpurun_out/pmc_*_$REC
echo done
