#!/bin/bash
# rocprofv3 kernel stats of the headline step under different environment settings, one profile per arm:
#   bash scripts/prof_ab.sh "NBP_GLDS=0" "-" ...   -> gpurun_out/prof_ab<i>/ ; compare with scripts/kstats_diff.py
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for arm in "$@"; do
  envs="$arm"
  [ "$envs" = "-" ] && envs=""
  for kv in $envs; do export "$kv"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ab$i -o run --output-format csv -- \
      python bench.py --steps 10 --warmup 2 --quick > gpurun_out/prof_ab$i.log 2>&1
  rc=$?
  for kv in $envs; do unset "${kv%%=*}"; done
  echo "arm $i [$arm] rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  i=$((i + 1))
done
exit 0
