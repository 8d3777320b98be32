#!/bin/bash
# A/B: eager vs graph replay, wgrad side-stream overlap on / off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for ov in 1 0; do
  for mode in "" "--eager"; do
    NBP_OVERLAP_WGRAD=$ov timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $mode > gpurun_out/ab_${ov}${mode}.log 2>&1 || exit $?
    echo "overlap=$ov mode=${mode:-graph}: $(grep -o '"value": [0-9.]*' gpurun_out/ab_${ov}${mode}.log)"
  done
done
