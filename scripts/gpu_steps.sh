#!/bin/bash
# One GPU session of named steps (STEPS, comma-separated), each under its own time limit; logs under gpurun_out/$OUT.
# Stops at the first crash / abort / timeout (exit codes other than 0 and 1); ordinary test failures continue.
#   STEPS=newtests,pytest,bench,rehearse OUT=r4a bash scripts/gpu_steps.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUT:-steps}
mkdir -p "$OUT"
: > "$OUT/summary.txt"
run() {
  local name=$1 t=$2
  shift 2
  local t0=$(date +%s)
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(( $(date +%s) - t0 ))s" | tee -a "$OUT/summary.txt"
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
PYT=(python -u -m pytest -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread)
STEPS=${STEPS:-smoke,pytest,bench}
[[ ,$STEPS, == *,smoke,* ]] && run smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
[[ ,$STEPS, == *,newtests,* ]] && run newtests 600 "${PYT[@]}" ${NEWTESTS:-tests/test_gpu_loss_api.py}
[[ ,$STEPS, == *,pytest,* ]] && run pytest_gpu 1000 "${PYT[@]}" tests -m gpu
[[ ,$STEPS, == *,bench,* ]] && run bench 400 python bench.py --quick --steps 10 --warmup 3
[[ ,$STEPS, == *,benchfull,* ]] && run benchfull 900 python bench.py
[[ ,$STEPS, == *,rehearse,* ]] && run rehearse 400 env NBP_BENCH_REHEARSE=1 python bench.py --gpus 2 --quick --steps 5 --warmup 2
[[ ,$STEPS, == *,extra,* ]] && run extra 600 ${EXTRA}
[[ ,$STEPS, == *,extra2,* ]] && run extra2 600 ${EXTRA2}
[[ ,$STEPS, == *,extra3,* ]] && run extra3 600 ${EXTRA3}
exit 0
