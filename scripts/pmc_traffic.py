"""HBM traffic per launch from the two PMC passes of scripts/pmc_pass.sh (MI355X_MICROARCH.md, HBM section):
bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 — FETCH_SIZE / WRITE_SIZE are in KiB and gfx950's FETCH_SIZE reports
half the bytes of wide coalesced reads.  Writes profiles/<out>.json keyed by bench.py's kernel classes.

    python scripts/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write profiles/r01_pmc_traffic.json
"""
import collections
import csv
import json
import sys

CLASSES = {"gemm_bf16": "gemm_bf16_kernel", "wgrad_f32": "wgrad_", "gemm_f32": "gemm_f32_kernel",
           "dw_bwd": "dw_bwd_tiled", "dw_fwd": "dw_sg_pool_tiled", "ln_fwd": "ln_fwd_nhwc", "ln_bwd": "ln_bwd_nhwc"}


def load(d, counter):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if r["Counter_Name"] == counter:
            per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return per


def main(fetch_dir, write_dir, out):
    f, w = load(fetch_dir, "FETCH_SIZE"), load(write_dir, "WRITE_SIZE")
    res = {"method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes (--kernel-trace --stats), "
                     "bench.py --eager --steps 3 --warmup 1; bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 per launch",
           "classes": {}}
    for cls, pat in CLASSES.items():
        names = [k for k in f if pat in k]
        n = sum(len(f[k]) for k in names)
        if not n:
            continue
        fetch = sum(sum(f[k]) for k in names) * 1024.0
        write = sum(sum(w.get(k, [])) for k in names) * 1024.0
        res["classes"][cls] = {"launches": n, "fetch_size_bytes_raw": fetch / n, "write_bytes": write / n,
                               "traffic_bytes_per_launch": (2 * fetch + write) / n}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res["classes"], indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
