#!/bin/bash
# Kernel-trace stats of the middle-level grouped weight gradient (scripts/wgroup_micro.py) per variant: the group
# kernel's and the slab reductions' average durations.  VARIANTS: comma-separated env assignments per variant.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/wgroup_trace
mkdir -p $O
: > $O/summary.txt
i=0
for v in ${VARIANTS:-NBP_WGRAD_GLDS=3 NBP_WGRAD_GLDS=43}; do
  i=$((i + 1))
  env ${v//,/ } REPS=20 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/t$i -o run --output-format csv \
      -- python scripts/wgroup_micro.py > $O/t$i.log 2>&1 || exit 1
  echo "== $v: $(grep -h 'per group' $O/t$i.log)" >> $O/summary.txt
  python - "$O/t$i" >> $O/summary.txt <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if "wgrad" in n or "reduce" in n:
        print(f"  {float(r['AverageNs']) / 1e3:8.1f} us  n={r['Calls']:>4}  {n[:90]}")
PY
done
cat $O/summary.txt
