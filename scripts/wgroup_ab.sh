#!/bin/bash
# Grouped weight-gradient variants (NBP_WGRAD_GLDS) on the middle and 32x32 levels' groups (scripts/wgroup_micro.py),
# alternated twice; then the --quick bench for the default and the given variants.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/wgroup_ab.txt
: > $out
for rep in 1 2; do
  for v in ${VARIANTS:-3 43 44}; do
    for lvl in "WG_C=512 WG_HW=256 WG_BLOCKS=6" "WG_C=256 WG_HW=1024 WG_BLOCKS=5" "WG_C=128 WG_HW=4096 WG_BLOCKS=3"; do
      echo -n "NBP_WGRAD_GLDS=$v $lvl: " >> $out
      env NBP_WGRAD_GLDS=$v $lvl timeout -k 10 120 python scripts/wgroup_micro.py >> $out 2>&1 || exit 1
    done
  done
done
for v in ${BENCH_VARIANTS:-3 44}; do
  echo -n "bench NBP_WGRAD_GLDS=$v: " >> $out
  env NBP_WGRAD_GLDS=$v timeout -k 10 300 python bench.py --quick --steps 20 --warmup 5 2>/dev/null | grep -o '"value": [0-9.]*' >> $out || exit 1
done
cat $out
