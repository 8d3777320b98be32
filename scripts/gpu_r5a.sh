#!/bin/bash
# Round-5 check session: the new / changed GPU tests, then the default bench line (headline + modes + cfg3 + cfg4 +
# cfg5 + CPU baseline).  Each GPU step has its own time limit; the script stops at the first failure.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r5a
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "${K:-lpips_against_float64 or cfg5_training or rehearsal_line}" > gpurun_out/r5a/pytest.log 2>&1 \
    || { tail -40 gpurun_out/r5a/pytest.log; exit 1; }
tail -5 gpurun_out/r5a/pytest.log
grep -h "near-ties" gpurun_out/r5a/pytest.log || true
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/r5a/bench.json 2> gpurun_out/r5a/bench.err
  tail -c 1500 gpurun_out/r5a/bench.json
fi
