#!/bin/bash
# The stage flushes of one eager cfg2 step: descriptors (NBP_REDUCE_LOG) and reduce_multi_kernel durations (rocprofv3
# kernel trace), in launch order.  Output: gpurun_out/reduce_probe/{log.txt,durations.txt}
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/reduce_probe
mkdir -p $O
NBP_REDUCE_LOG=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- \
    python bench.py --steps 1 --warmup 1 --quick --eager > $O/bench.json 2> $O/stderr.txt
grep "\[reduce\]" $O/stderr.txt > $O/log.txt || true
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/reduce_probe/prof/**/run_kernel_trace.csv", recursive=True) or glob.glob("gpurun_out/reduce_probe/prof/run_kernel_trace.csv")
rows = list(csv.DictReader(open(f[0])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
out = [f'{(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3:.1f}' for r in rows if "reduce_multi_kernel" in r["Kernel_Name"]]
open("gpurun_out/reduce_probe/durations.txt", "w").write("\n".join(out) + "\n")
print(len(out), "reduce launches")
PY
rm -rf $O/prof
