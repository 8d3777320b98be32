"""HBM traffic and MFMA busy per launch from the PMC passes of scripts/pmc_pass.sh (MI355X_MICROARCH.md, HBM and PMC
sections): bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 -- FETCH_SIZE / WRITE_SIZE are in KiB and gfx950's FETCH_SIZE
reports half the bytes of wide coalesced reads; MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (dispatch ns * 2.4 GHz * 1024
SIMDs) (the counter sums MFMA-pipe cycles over the SIMDs, ~32 per v_mfma_f32_32x32x16 -- calibrated against the GEMM
class's algorithmic MFMA count; 2.4 GHz is the peak clock, so this is a lower bound on utilisation; rocprofv3 reports
GRBM_GUI_ACTIVE summed over the 8 XCDs, so it is not used as the denominator) and MFMA FLOP rate = (MOPS_F16 + MOPS_BF16
+ MOPS_F32) * 512 / dispatch ns vs the dense peak of the dtype.  Writes profiles/<out>.json keyed by bench.py's kernel
classes.

    python scripts/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_mfma profiles/rNN_pmc_traffic.json
"""
import collections
import csv
import json
import os
import re
import sys

CLASSES = {"gemm16": ("gemm_glds_kernel", "gemm_bf16_kernel", "gemm_skinny_kernel"), "gemm_f32": ("gemm_f32_kernel",),
           # weight gradients launched at once (N or K <= 64) / the grouped wide launches of a U-Net level, and the
           # fp32 slab reductions (+ layer-scale post-ops) that fold their split-M partials: per KERNEL launch, the
           # unit bench.py's algorithmic bytes use for these classes
           "wgrad_narrow": ("wgrad_bf16_kernel", "wgrad_f32_kernel", "wgrad_narrow_full"), "wgrad_group": ("wgrad_bf16_wide",),
           "reduce": ("reduce_multi_kernel", "reduce_table_kernel", "layer_scale_grad_kernel"),
           "dw_bwd": ("dw_bwd_tiled",), "dw_bwd_32": (re.compile(r"dw_bwd_tiledI\w+?Lb1ELi32E(Lb0E)?E"),),
           "dw_bwd_sca_32": (re.compile(r"dw_bwd_tiledI\w+?Lb1ELi32ELb1EE"),),
           "dw_bwd_sca_16": (re.compile(r"dw_bwd_tiledI\w+?Lb1ELi16ELb1EE"),),
           "dw_fwd": ("dw_sg_pool_tiled",), "c1dw": ("c1_dw_sg_pool_img",), "ln_fwd": ("ln_fwd_nhwc",),
           "c1dw_tile_fwd": ("c1dw_fwd_tile",), "c1dw_tile_bwd": ("c1dw_bwd_tile",),
           # bench.py's one-instance classes (INSTANCES / ROCPROF_KERNELS there)
           "c1dw_bwd_L0": (re.compile(r"c1dw_bwd_tileI\w+?Li32ELi\d+ELb[01]E(Lb0E)?E"),),
           "c1dw_bwd_L1": (re.compile(r"c1dw_bwd_tileI\w+?Li64ELi\d+ELb[01]E(Lb0E)?E"),),
           "c1dw_bwd_sca_L0": (re.compile(r"c1dw_bwd_tileI\w+?Li32ELi\d+ELb[01]ELb1EE"),),
           "c1dw_bwd_sca_L1": (re.compile(r"c1dw_bwd_tileI\w+?Li64ELi\d+ELb[01]ELb1EE"),),
           "dw_bwd_16": (re.compile(r"dw_bwd_tiledI\w+?Lb1ELi16E(Lb0E)?E"),),
           "wgrad_group_512": (re.compile(r"wgrad_bf16_wide_groupI\w+?Li3ELi512ELi2EE"),),
           "wgrad_group_768": (re.compile(r"wgrad_bf16_wide_groupI\w+?Li3ELi768ELi4EE"),),
           "reduce_multi": ("reduce_multi_kernel",), "reduce_table": ("reduce_table_kernel",),
           "layer_scale_grad": ("layer_scale_grad_kernel",),
           "ffn_rows": ("ffn_rows_fwd", "ffn_rows_bwd"),
           "ffn_rows_bwd_512": (re.compile(r"ffn_rows_bwdI\w+?Li512ELb0EE"),),
           "ffn_rows_bwd_256": (re.compile(r"ffn_rows_bwdI\w+?Li256ELb0EE"),),
           "ffn_rows_bwd_128": (re.compile(r"ffn_rows_bwdI\w+?Li128ELb0EE"),),
           "ffn_rows_bwd_pre_512": (re.compile(r"ffn_rows_bwdI\w+?Li512ELb1EE"),),
           "ffn_rows_bwd_pre_256": (re.compile(r"ffn_rows_bwdI\w+?Li256ELb1EE"),),
           "ffn_rows_bwd_pre_128": (re.compile(r"ffn_rows_bwdI\w+?Li128ELb1EE"),),
           "ffn_rows_512": (re.compile(r"ffn_rows_fwdI\w+?Li512EE"),),
           "ffn_rows_256": (re.compile(r"ffn_rows_fwdI\w+?Li256EE"),), "ffn_rows_128": (re.compile(r"ffn_rows_fwdI\w+?Li128EE"),),
           "ln_bwd": ("ln_bwd_nhwc",),
           # VGG / AlexNet implicit-GEMM convs (cfg3's perceptual + LPIPS trunks): the tiled kernels with A mode 3 / 4
           "vgg_conv": (re.compile(r"gemm_(glds|bf16)_kernelILi\d+ELi\d+ELi\d+ELi[34]E"),),
           # the 256 x 256 DMA tiles of the N >= 256 VGG layers (a subset of vgg_conv)
           "vgg_conv_256": (re.compile(r"gemm_glds_kernelILi256ELi256ELi\d+ELi3E"),)}


def _match(name, pats):
    return any(p.search(name) if hasattr(p, "search") else p in name for p in pats)
SIMDS = 256 * 4


def load(d, counter, with_ns=False):
    per = collections.defaultdict(list)
    path = f"{d}/run_counter_collection.csv"
    if not os.path.exists(path):
        return per
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            v = float(r["Counter_Value"])
            per[r["Kernel_Name"]].append((v, int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) if with_ns else v)
    return per


CLOCK_GHZ = 2.4
PEAK = {"f16": 2.5e15, "bf16": 2.5e15, "f32": 157.3e12}


def main(fetch_dir, write_dir, mfma_dir, out):
    f, w = load(fetch_dir, "FETCH_SIZE"), load(write_dir, "WRITE_SIZE")
    mb = load(mfma_dir, "SQ_VALU_MFMA_BUSY_CYCLES", with_ns=True)
    mops = {t: load(mfma_dir, f"SQ_INSTS_VALU_MFMA_MOPS_{t.upper()}") for t in ("f16", "bf16", "f32")}
    res = {"method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE / --pmc SQ_VALU_MFMA_BUSY_CYCLES "
                     "SQ_INSTS_VALU_MFMA_MOPS_{F16,BF16,F32} in separate passes (--kernel-trace --stats), bench.py "
                     "--eager --quick --steps 3 --warmup 1; bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 per launch; "
                     f"mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (dispatch ns * {CLOCK_GHZ} GHz * 1024 SIMDs); "
                     "mfma_flops = MOPS * 512",
           "classes": {}}
    for cls, pats in CLASSES.items():
        names = [k for k in f if _match(k, pats)]
        n = sum(len(f[k]) for k in names)
        if not n:
            continue
        fetch = sum(sum(f[k]) for k in names) * 1024.0
        write = sum(sum(w.get(k, [])) for k in names) * 1024.0
        rec = {"launches": n, "fetch_size_bytes_raw": fetch / n, "write_bytes": write / n,
               "traffic_bytes_per_launch": (2 * fetch + write) / n}
        mn = [k for k in mb if _match(k, pats)]
        if mn:
            busy = sum(v for k in mn for v, _ in mb[k])
            ns = sum(t for k in mn for _, t in mb[k])
            nl = sum(len(mb[k]) for k in mn)
            rec.update({"mfma_busy_cycles_per_launch": busy / nl, "dispatch_us_per_launch": ns / nl / 1e3,
                        "mfma_busy_frac": busy / (ns * CLOCK_GHZ * SIMDS) if ns else None})
            for t, per in mops.items():
                fl = sum(sum(per.get(k, [])) for k in mn) * 512.0
                if fl:
                    rec[f"mfma_{t}_flops_per_launch"] = fl / nl
                    rec[f"mfma_{t}_flops_frac"] = fl / (ns * 1e-9) / PEAK[t]
        res["classes"][cls] = rec
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res["classes"], indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:5])
