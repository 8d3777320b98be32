#!/bin/bash
# Loader-wave GEMM tiles (NBP_GEMM_LW) A/B: the deep-level GEMM shapes (scripts/deep_gemm_probe.py) alternated twice,
# then the --quick bench per variant.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/gemm_lw_ab.txt
: > $out
for rep in 1 2; do
  for v in ${LW_VARIANTS:-0 1 2}; do
    env NBP_GEMM_LW=$v timeout -k 10 120 python scripts/deep_gemm_probe.py 2>/dev/null >> $out || exit 1
  done
done
for v in ${LW_BENCH:-0 1 2 0}; do
  echo -n "bench NBP_GEMM_LW=$v: " >> $out
  env NBP_GEMM_LW=$v timeout -k 10 300 python bench.py --quick --steps 20 --warmup 5 2>/dev/null | grep -o '"value": [0-9.]*' >> $out || exit 1
done
cat $out
