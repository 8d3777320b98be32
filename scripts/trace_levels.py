"""Per-level breakdown of ONE training step from a rocprofv3 kernel-trace CSV (graph replays included).

    python scripts/trace_levels.py <kernel_trace.csv> [top]

A step is the window from an `intro_fwd` launch to the next `adamw` launch; the last complete window is used (the
bench's timed HIP-graph replays come last).  The window is cut into segments at the U-Net level changes: the
down/up GEMMs (space-to-depth A-mode 1 / depth-to-space C-mode 1 of the tiled GEMM kernels, in both directions).  For
each segment: launches, busy time (sum of kernel durations), span (wall) and the gap share, plus its top kernels.
"""
import collections
import csv
import re
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("_ZN12_GLOBAL__N_1", "")
    m = re.match(r"\d+([a-z_0-9]+?)I(.*)E[Ev]", n)
    if m:
        return m.group(1) + "<" + ",".join(re.findall(r"Li(\d+)E", m.group(2))) + ">"
    return n.split("(")[0][:70]


def is_level_cut(name):
    if "gemm_bf16_kernel" not in name and "gemm_glds_kernel" not in name and "gemm_f32_kernel" not in name:
        return False
    a = [int(v) for v in re.findall(r"Li(\d+)E", name)]
    return len(a) >= 5 and (a[3] == 1 or a[4] == 1)


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    starts = [i for i, k in enumerate(ks) if "intro_fwd" in k[2]]
    win = None
    for s in reversed(starts):
        e = next((j for j in range(s, len(ks)) if "adamw" in ks[j][2]), None)
        if e is not None:
            win = ks[s:e + 1]
            break
    if win is None:
        sys.exit("no complete step window")
    span = (win[-1][1] - win[0][0]) / 1e6
    busy = sum(k[1] - k[0] for k in win) / 1e6
    print(f"step: {len(win)} launches, span {span:.3f} ms, busy {busy:.3f} ms, gaps {span - busy:.3f} ms")
    segs, cur = [], []
    for k in win:
        if is_level_cut(k[2]) and cur:
            segs.append(cur)
            cur = []
        cur.append(k)
    segs.append(cur)
    for i, sg in enumerate(segs):
        sp = (sg[-1][1] - sg[0][0]) / 1e6
        bz = sum(k[1] - k[0] for k in sg) / 1e6
        agg = collections.defaultdict(lambda: [0, 0.0])
        for k in sg:
            a = agg[short(k[2])]
            a[0] += 1
            a[1] += (k[1] - k[0]) / 1e3
        print(f"\nseg {i:2d}: {len(sg):4d} launches  span {sp:7.3f} ms  busy {bz:7.3f} ms  "
              f"({len(sg) and (sp - bz) / len(sg) * 1e3:.2f} us gap/launch)  first={short(sg[0][2])}")
        for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
            print(f"      {t / 1e3:7.3f} ms  n={c:4d}  avg={t / c:7.1f} us  {n}")
    agg = collections.defaultdict(lambda: [0, 0.0])
    for k in win:
        a = agg[short(k[2])]
        a[0] += 1
        a[1] += (k[1] - k[0]) / 1e3
    print("\nwhole step:")
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:30]:
        print(f"  {t / 1e3:7.3f} ms  n={c:4d}  avg={t / c:7.1f} us  {n}")


if __name__ == "__main__":
    main()
