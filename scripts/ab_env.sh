#!/bin/bash
# Interleaved A/B of environment settings on the quick bench (one gpurun session):
#   bash scripts/ab_env.sh OUT "ENV_A" "ENV_B" [...]   (each ENV a space-separated list of VAR=value, "-" for none)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$1
shift
mkdir -p gpurun_out/$OUT
ROUNDS=${ROUNDS:-2}
for r in $(seq $ROUNDS); do
  i=0
  for e in "$@"; do
    i=$((i + 1))
    envs=""
    [ "$e" != "-" ] && envs="$e"
    env $envs timeout -k 10 300 python bench.py --quick --steps ${STEPS:-20} --warmup 5 > gpurun_out/$OUT/ab_${i}_r$r.json 2> gpurun_out/$OUT/ab_${i}_r$r.err || exit $?
    v=$(python -c "import json,sys;d=json.load(open('gpurun_out/$OUT/ab_${i}_r$r.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['frac'])")
    echo "round $r  [$e]  $v" | tee -a gpurun_out/$OUT/ab.txt
  done
done
