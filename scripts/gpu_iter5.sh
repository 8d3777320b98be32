#!/bin/bash
# Round-5 iteration session: selected GPU tests (K), the level-0/1 tile micro-benchmark, a quick bench line.
# Each GPU step has its own time limit; the script stops at the first failure.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-it5}
mkdir -p $O
export TMPDIR=/tmp
if [ -n "${K:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
      -k "$K" > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
  tail -3 $O/pytest.log
  grep -h "branch decisions" $O/pytest.log || true
fi
if [ "${MICRO:-1}" = 1 ]; then
  timeout -k 10 300 python -u scripts/c1dw_tile_micro.py 20 > $O/micro.txt 2>&1 || { tail -30 $O/micro.txt; exit 1; }
  cat $O/micro.txt
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 300 python bench.py --quick --steps 20 --warmup 5 ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('value', d['value'], 'ms', d['ms_per_step'], 'nafblock', d['nafblock_roofline']['frac'], d['nafblock_roofline']['per_level_eager'])"
fi
