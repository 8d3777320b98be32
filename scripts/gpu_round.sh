#!/bin/bash
# One measurement session on the GPU box: the default bench line (headline + modes + cfg3 + CPU baseline), a
# rocprofv3 kernel-trace/stats profile of the quick bench, and the PMC passes (traffic + MFMA busy).  Each GPU step
# has its own time limit; the script stops at the first failure.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "cpus: os.cpu_count=$(python -c 'import os;print(os.cpu_count())') affinity=$(python -c 'import os;print(len(os.sched_getaffinity(0)))') nproc=$(nproc)" | tee gpurun_out/host.txt
grep -m1 "model name" /proc/cpuinfo | tee -a gpurun_out/host.txt
[[ ${STEPS:-bench,prof,pmc} == *bench* ]] && timeout -k 10 600 python bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err && tail -c 600 gpurun_out/bench.log
if [[ ${STEPS:-bench,prof,pmc} == *prof* ]]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
      python bench.py --steps 10 --warmup 3 --quick > gpurun_out/prof_bench.log 2>&1
  ls gpurun_out/prof
fi
if [[ ${STEPS:-bench,prof,pmc} == *pmc* ]]; then
  timeout -s KILL 30 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
  bash scripts/pmc_pass.sh
fi
