#!/bin/bash
# A/B of two builds of the library: the in-tree one and lowlight_image_enhancement_amd/_lib/ab/liblowlight_nbp.so
# (a variant linked by hand, selected with NBP_LIB).  Deep-level GEMM probe and the --quick bench, arms alternated.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/ab_lib.txt
: > $out
B="NBP_LIB=$PWD/lowlight_image_enhancement_amd/_lib/ab/liblowlight_nbp.so"
for arm in "" "$B"; do
  echo "== probe ${arm:+variant}${arm:-in-tree}" >> $out
  env $arm timeout -k 10 120 python scripts/deep_gemm_probe.py >> $out 2>&1 || exit 1
done
for rep in 1 2; do
  for arm in "" "$B"; do
    echo "== bench ${arm:+variant}${arm:-in-tree}" >> $out
    env $arm timeout -k 10 300 python bench.py --quick --steps 20 --warmup 5 2>/dev/null | grep -o '"value": [0-9.]*' >> $out || exit 1
  done
done
