#!/bin/bash
# A/B of the level-0/1 tile path in the quick bench: none / level 0 only / level 1 only / both (interleaved twice).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-ab}
mkdir -p $O
for rep in 1 2; do
  for tc in "" 32 64 32,64; do
    NBP_C1DW_TILE_C=$tc timeout -k 10 300 python bench.py --quick --steps 20 --warmup 5 > $O/b_${rep}_${tc:-none}.json 2> $O/b.err || { tail -30 $O/b.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_${rep}_${tc:-none}.json').read().strip().splitlines()[-1]); print('tile_c=${tc:-none}', d['value'], d['ms_per_step'], {k: (v['fwd_ms'], v['bwd_ms']) for k, v in d['nafblock_roofline']['per_level_eager'].items() if 'C32' in k or 'C64' in k})"
  done
done
