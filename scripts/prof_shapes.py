"""Per-(kernel, grid) time per step from a rocprofv3 kernel_trace CSV: python scripts/prof_shapes.py <csv> <steps> [substr ...]"""
import collections
import csv
import sys

path, steps = sys.argv[1], int(sys.argv[2])
keys = sys.argv[3:]
agg = collections.defaultdict(lambda: [0, 0.0])
for r in csv.DictReader(open(path)):
    n = r["Kernel_Name"]
    if keys and not any(k in n for k in keys):
        continue
    g = (int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
    a = agg[(n[:60], g, int(r["Workgroup_Size_X"]))]
    a[0] += 1
    a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
    print(f"{v[1] / steps:8.1f} us/step  n/step={v[0] / steps:5.1f} avg={v[1] / v[0]:7.1f}us  blocks={k[1]} wg={k[2]}  {k[0]}")
