#!/bin/bash
# Iteration loop on the GPU box: GPU parity tests, then the bench under a rocprofv3 kernel trace (the bench JSON line
# lands in gpurun_out/it_bench.log, the per-dispatch trace in gpurun_out/it/run_kernel_trace.csv; analyse it with
# scripts/trace_levels.py).  Stops at the first failure.  TESTS=0 skips the tests, K selects pytest -k.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
      ${K:+-k "$K"} > gpurun_out/it_pytest.log 2>&1 || { tail -30 gpurun_out/it_pytest.log; exit 1; }
  tail -2 gpurun_out/it_pytest.log
fi
rm -rf gpurun_out/it
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/it -o run --output-format csv -- \
    python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/it_bench.log 2>&1
tail -1 gpurun_out/it_bench.log | cut -c1-400
