#!/bin/bash
# A/B of the channel-dot load batching against lowlight_image_enhancement_amd/_lib/ab/old.so: bit pins written by
# the old build and checked on the new one, the --quick bench (arms alternated).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/ab_chandot.txt
: > $out
OLD="NBP_LIB=$PWD/lowlight_image_enhancement_amd/_lib/ab/old.so"
env $OLD timeout -k 10 120 python tests/test_gpu_chandot_bits.py --write >> $out 2>&1 || { tail -30 $out; exit 1; }
cp tests/golden/chandot_bits_sha.json gpurun_out/chandot_bits_sha.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_chandot_bits.py tests/test_gpu_parity.py -k "chandot or sca or chan" -x -q --timeout 120 --timeout-method thread >> $out 2>&1 || { tail -30 $out; exit 1; }
for arm in "$OLD" ""; do
  echo "== chandot_time ${arm:+old}${arm:-new}" >> $out
  env $arm timeout -k 10 120 python scripts/chandot_time.py >> $out 2>&1 || exit 1
done
for rep in 1 2; do
  for arm in "$OLD" ""; do
    echo "== bench ${arm:+old}${arm:-new}" >> $out
    env $arm timeout -k 10 300 python bench.py --quick --steps 20 --warmup 5 2>/dev/null | grep -o '"value": [0-9.]*' >> $out || exit 1
  done
done
cat $out | grep -v amdgpu.ids
