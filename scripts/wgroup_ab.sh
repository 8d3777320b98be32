#!/bin/bash
# Grouped weight-gradient variants on the middle, 32x32 and 64x64 levels' groups (scripts/wgroup_micro.py),
# alternated twice; then the --quick bench per bench variant.  A variant is a comma-separated list of environment
# assignments, e.g. VARIANTS="NBP_WGRAD_GLDS=3 NBP_WGRAD_GLDS=43,NBP_WGROUP_XCD=0".
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/wgroup_ab.txt
: > $out
VARIANTS=${VARIANTS:-NBP_WGRAD_GLDS=3 NBP_WGRAD_GLDS=43 NBP_WGRAD_GLDS=44}
for rep in 1 2; do
  for v in $VARIANTS; do
    for lvl in "WG_C=512 WG_HW=256 WG_BLOCKS=6" "WG_C=256 WG_HW=1024 WG_BLOCKS=5" "WG_C=128 WG_HW=4096 WG_BLOCKS=3"; do
      echo -n "$v $lvl: " >> $out
      env ${v//,/ } $lvl timeout -k 10 120 python scripts/wgroup_micro.py >> $out 2>&1 || exit 1
    done
  done
done
for v in ${BENCH_VARIANTS:-NBP_WGRAD_GLDS=3 NBP_WGRAD_GLDS=43}; do
  echo -n "bench $v: " >> $out
  env ${v//,/ } timeout -k 10 300 python bench.py --quick --steps 20 --warmup 5 2>/dev/null | grep -o '"value": [0-9.]*' >> $out || exit 1
done
cat $out
