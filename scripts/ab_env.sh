#!/bin/bash
# A/B of an executor switch in the quick bench: AB_VAR takes each of AB_VALS in turn (interleaved, REPS times), e.g.
#   AB_VAR=NBP_LN_WG AB_VALS="1 0" scripts/ab_env.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-ab}
mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do
  for v in $AB_VALS; do
    t=$(basename "$v")  # (a path value, e.g. NBP_LIB=<an A/B build>)
    env "$AB_VAR=$v" timeout -k 10 300 python bench.py --quick --steps 20 --warmup 5 > $O/b_${rep}_$t.json 2> $O/b.err || { tail -30 $O/b.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_${rep}_$t.json').read().strip().splitlines()[-1]); print('$AB_VAR=$t', d['value'], d['ms_per_step'], {k: (v['fwd_ms'], v['bwd_ms']) for k, v in d['nafblock_roofline']['per_level_eager'].items() if 'C32' in k})"
  done
done
