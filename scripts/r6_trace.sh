# rocprof kernel trace + stats of the quick fp16 cfg2 bench, per-level breakdown (scripts/trace_levels.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r6_trace}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tmp -o run --output-format csv -- \
    python bench.py --steps 10 --warmup 3 --quick > $O/prof_bench.json 2> $O/prof_bench_stderr.txt || exit $?
cp gpurun_out/prof_tmp/run_kernel_stats.csv $O/kernel_stats.csv
python scripts/trace_levels.py gpurun_out/prof_tmp/run_kernel_trace.csv > $O/trace_levels.txt
rm -rf gpurun_out/prof_tmp
head -3 $O/trace_levels.txt
