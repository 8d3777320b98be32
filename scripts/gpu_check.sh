#!/bin/bash
# One GPU session: smoke -> GPU parity tests -> bench -> rocprofv3 kernel stats.
# Stops at the first crash / abort / timeout (exit codes other than 0 and 1); ordinary test failures continue.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/summary.txt
run() {
  local name=$1 t=$2
  shift 2
  local t0=$(date +%s)
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(( $(date +%s) - t0 ))s" | tee -a gpurun_out/summary.txt
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-smoke,pytest,bench,prof}
[[ $STEPS == *smoke* ]] && run smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
KARGS=()
[ -n "${PYTEST_K:-}" ] && KARGS=(-k "$PYTEST_K")
[[ $STEPS == *pytest* ]] && run pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread "${KARGS[@]}"
[[ $STEPS == *bench* ]] && run bench 600 python bench.py --steps 10 --warmup 3
if [[ $STEPS == *prof* ]]; then
  export TMPDIR=/tmp
  run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
      python bench.py --steps 5 --warmup 2 --no-cpu-baseline
fi
exit 0
