#!/bin/bash
# One iteration on the GPU box: GPU test suite (optionally filtered by PYTEST_K), the depthwise per-level timings and
# a quick bench line.  Each GPU step has its own time limit; the script stops at the first crash / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local name=$1 t=$2
  shift 2
  local t0=$(date +%s)
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(( $(date +%s) - t0 ))s" | tee -a gpurun_out/summary.txt
  tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
: > gpurun_out/summary.txt
STEPS=${STEPS:-pytest,dw,bench}
KARGS=()
[ -n "${PYTEST_K:-}" ] && KARGS=(-k "$PYTEST_K")
[[ $STEPS == *pytest* ]] && run pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread "${KARGS[@]}"
[[ $STEPS == *dw* ]] && run dw_time 300 python scripts/dw_time.py
[[ $STEPS == *bench* ]] && run bench 600 python bench.py --quick --steps 20 --warmup 5
[[ $STEPS == *barrier* ]] && run xcd_barrier 120 build/xcd_barrier_probe
exit 0
