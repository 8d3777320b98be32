#!/bin/bash
# A/B bench runs under different environment settings: bash scripts/ab_env.sh "VAR=a" "VAR=b" ...
# ("-" = defaults; "EAGER" or "EAGER:VAR=x" = the --eager launch mode).  Prints value / ms_per_step per arm into gpurun_out/ab.txt.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ab.txt
for arm in "$@"; do
  extra=""
  envs="${arm#EAGER}"
  envs="${envs#:}"
  [ "$envs" = "-" ] && envs=""
  [[ "$arm" == EAGER* ]] && extra="--eager"
  env $envs timeout -k 10 300 python bench.py --steps 20 --warmup 3 --quick $extra > gpurun_out/ab_last.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$arm rc=$rc" | tee -a gpurun_out/ab.txt; tail -5 gpurun_out/ab_last.log; exit $rc; fi
  grep '^{' gpurun_out/ab_last.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$arm', d['value'], d['ms_per_step'])" | tee -a gpurun_out/ab.txt
done
