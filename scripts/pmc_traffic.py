"""HBM traffic and MFMA busy per launch from the PMC passes of scripts/pmc_pass.sh (MI355X_MICROARCH.md, HBM and PMC
sections): bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 -- FETCH_SIZE / WRITE_SIZE are in KiB and gfx950's FETCH_SIZE
reports half the bytes of wide coalesced reads; MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE * 1024 SIMDs)
(the counter counts MFMA-pipe cycles summed over SIMDs, 32 per v_mfma_f32_32x32x16; GRBM_GUI_ACTIVE = the dispatch's GPU
cycles).  Writes profiles/<out>.json keyed by bench.py's kernel classes.

    python scripts/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_mfma profiles/rNN_pmc_traffic.json
"""
import collections
import csv
import json
import os
import sys

CLASSES = {"gemm16": ("gemm_bf16_kernel", "gemm_skinny_kernel"), "wgrad": ("wgrad_",), "gemm_f32": ("gemm_f32_kernel",),
           "dw_bwd": ("dw_bwd_tiled",), "dw_fwd": ("dw_sg_pool_tiled",), "ln_fwd": ("ln_fwd_nhwc",),
           "ln_bwd": ("ln_bwd_nhwc",)}
SIMDS = 256 * 4


def load(d, counter):
    per = collections.defaultdict(list)
    path = f"{d}/run_counter_collection.csv"
    if not os.path.exists(path):
        return per
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return per


def main(fetch_dir, write_dir, mfma_dir, out):
    f, w = load(fetch_dir, "FETCH_SIZE"), load(write_dir, "WRITE_SIZE")
    mb, ga = load(mfma_dir, "SQ_VALU_MFMA_BUSY_CYCLES"), load(mfma_dir, "GRBM_GUI_ACTIVE")
    bc = load(mfma_dir, "SQ_BUSY_CU_CYCLES")
    res = {"method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE / --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES "
                     "GRBM_GUI_ACTIVE in separate passes (--kernel-trace --stats), bench.py --eager --quick --steps 3 "
                     "--warmup 1; bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 per launch; mfma_busy = "
                     "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE * 1024 SIMDs)",
           "classes": {}}
    for cls, pats in CLASSES.items():
        names = [k for k in f if any(p in k for p in pats)]
        n = sum(len(f[k]) for k in names)
        if not n:
            continue
        fetch = sum(sum(f[k]) for k in names) * 1024.0
        write = sum(sum(w.get(k, [])) for k in names) * 1024.0
        rec = {"launches": n, "fetch_size_bytes_raw": fetch / n, "write_bytes": write / n,
               "traffic_bytes_per_launch": (2 * fetch + write) / n}
        mn = [k for k in mb if any(p in k for p in pats)]
        if mn:
            busy = sum(sum(mb[k]) for k in mn)
            gui = sum(sum(ga.get(k, [])) for k in mn)
            rec.update({"mfma_busy_cycles_per_launch": busy / sum(len(mb[k]) for k in mn),
                        "gpu_cycles_per_launch": gui / max(sum(len(ga.get(k, [])) for k in mn), 1),
                        "busy_cu_cycles_per_launch": sum(sum(bc.get(k, [])) for k in mn) / max(
                            sum(len(bc.get(k, [])) for k in mn), 1),
                        "mfma_busy_frac": busy / (gui * SIMDS) if gui else None})
        res["classes"][cls] = rec
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res["classes"], indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:5])
