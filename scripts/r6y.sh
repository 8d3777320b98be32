set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=r6y bash scripts/r6_trace.sh || exit 1
O=gpurun_out/r6y_fp32
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tmp32 -o run --output-format csv -- \
    python bench.py --steps 4 --warmup 2 --quick --precision fp32 > $O/prof_bench.json 2> $O/prof_bench_stderr.txt || exit $?
cp gpurun_out/prof_tmp32/run_kernel_stats.csv $O/kernel_stats.csv
python scripts/trace_levels.py gpurun_out/prof_tmp32/run_kernel_trace.csv > $O/trace_levels.txt
rm -rf gpurun_out/prof_tmp32
head -1 $O/trace_levels.txt
