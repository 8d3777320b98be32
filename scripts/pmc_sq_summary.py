"""Per-kernel SQ counter summary of scripts/pmc_tile.sh passes (FETCH_SIZE in KiB summed over dispatches): per-wave averages (counters summed over the
dispatches of a kernel name, divided by its SQ_WAVES), cycle counters in quad-cycles as rocprofv3 reports them.
    python scripts/pmc_sq_summary.py gpurun_out/<tag>"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(os.path.join(d, "pmc_*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if not any(s in k for s in ("c1dw", "dw_bwd_tiled", "dw_sg_pool", "gemm_skinny", "gemm_glds", "wgrad", "reduce")):
            continue
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add((f, r.get("Dispatch_Id", "")))
for k, c in sorted(tot.items()):
    w = c.get("SQ_WAVES", 0) or 1
    name = k.split("(")[0][:90]
    print(name)
    print("  " + ", ".join(f"{n}={v / w:.0f}" for n, v in sorted(c.items()) if n not in ("SQ_WAVES", "FETCH_SIZE")) +
          f"  | waves={w:.0f} FETCH_SIZE(KiB, sum)={c.get('FETCH_SIZE', 0):.0f}")
