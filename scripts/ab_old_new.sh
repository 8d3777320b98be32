#!/bin/bash
# A/B of the in-tree library against lowlight_image_enhancement_amd/_lib/ab/old.so (the build before a kernel change,
# selected with NBP_LIB; or ARM_A="VAR=value" for a knob of the same build): bit pins written by the old build, checked on the new one; per-level depthwise timings and
# the --quick bench, arms alternated.  WRITE_GOLD=1 writes tests/golden/dw_bwd_sha.json from the old build first.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/ab_old_new.txt
: > $out
OLD="${ARM_A:-NBP_LIB=$PWD/lowlight_image_enhancement_amd/_lib/ab/old.so}"  # ARM_A: another env for the old arm
if [ "${WRITE_GOLD:-0}" = 1 ]; then
  env $OLD timeout -k 10 120 python tests/test_gpu_dw_bwd_bits.py --write >> $out 2>&1 || exit 1
  cp tests/golden/dw_bwd_sha.json gpurun_out/dw_bwd_sha.json
fi
timeout -k 10 300 python -u -m pytest tests/test_gpu_dw_bwd_bits.py ${EXTRA_TESTS:-} -x -q --timeout 120 --timeout-method thread >> $out 2>&1 || { tail -30 $out; exit 1; }
for arm in "$OLD" ""; do
  echo "== dw_time ${arm:+old}${arm:-new}" >> $out
  env $arm timeout -k 10 120 python scripts/dw_time.py >> $out 2>&1 || exit 1
done
for rep in 1 2; do
  for arm in "$OLD" ""; do
    echo "== bench ${arm:+old}${arm:-new}" >> $out
    env $arm timeout -k 10 300 python bench.py --quick --steps 20 --warmup 5 2>/dev/null | grep -o '"value": [0-9.]*' >> $out || exit 1
  done
done
cat $out | grep -v amdgpu.ids
