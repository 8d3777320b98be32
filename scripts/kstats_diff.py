"""Per-kernel time per step of two rocprofv3 --stats runs (scripts/prof_ab.sh arms):
python scripts/kstats_diff.py gpurun_out/prof_ab0 gpurun_out/prof_ab1 [steps]"""
import csv
import glob
import sys


def load(d):
    f = glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)[0]
    out = {}
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        key = n[n.find("N_1") + 3:][:70] if "N_1" in n else n[:70]
        a = out.setdefault(key, [0.0, 0])
        a[0] += float(r["TotalDurationNs"])
        a[1] += int(r["Calls"])
    return out


a, b = load(sys.argv[1]), load(sys.argv[2])
steps = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
keys = sorted(set(a) | set(b), key=lambda k: -(a.get(k, [0])[0] + b.get(k, [0])[0]))
ta = sum(v[0] for v in a.values()) / steps / 1e6
tb = sum(v[0] for v in b.values()) / steps / 1e6
print(f"total ms/step  A {ta:.3f}  B {tb:.3f}")
for k in keys[:40]:
    x, y = a.get(k, [0, 0]), b.get(k, [0, 0])
    print(f"{x[0] / steps / 1e6:7.3f} {y[0] / steps / 1e6:7.3f}  calls {x[1] / steps:6.1f} {y[1] / steps:6.1f}  {k}")
