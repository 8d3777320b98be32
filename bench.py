"""Benchmark: training images/sec of the NewBP-NAFNet hot path on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1], the 1-GPU headline config): NAFNet width 32, enc [2,2,4,8], middle 12,
dec [2,2,2,2] (29.16 M params), rgb/B2 crosstalk PSF, 16 x 3 x 256 x 256 synthetic sRGB per GPU,
HybridLoss terms L1 + SSIM + Phys_srgb, global-norm clip 0.01 + AdamW.  One "step" = forward + loss + backward
(+ bucketed RCCL all-reduce when N > 1) + clip + AdamW, all HIP kernels.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    (N > 1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...)

Rank 0 prints ONE JSON line.  `roofline` is the dominant kernel class measured live with HIP events on the launch
stream during the timed steps; `nafblock_roofline` is the north-star figure (NAFBlock fwd+bwd algorithmic bytes,
SURVEY §8d: 5*B*C*H*W*4 bytes per block per step, vs 8 TB/s); `cpu_baseline` is the CPU oracle (oracle/, kind
"port") on a bounded sample, timed on this box's host cores; `psnr_vs_cpu_ref_db` compares the GPU output with
the CPU oracle's on the same weights and input.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "training images/sec at 256×256 bs=16 (1/2/4/8 GPU) + PSNR vs CPU ref"
CFG = dict(width=32, enc_blk_nums=[2, 2, 4, 8], middle_blk_num=12, dec_blk_nums=[2, 2, 2, 2])
# BASELINE.json configs[1] (the headline) and configs[2] (VGG19 perceptual + LPIPS + ΔE00, bs8 512²; weights from
# configs/colab/sid_newbp_rgb.yml:78-96; LPIPS is the HybridLossPlus term's net='vgg', synthetic offline weights)
WORKLOADS = {
    "cfg2": dict(batch=16, img=256, w=dict(w_l1=1.0, w_ssim=0.05, w_phys=0.1),
                 desc="cfg2: NAFNet w32 enc[2,2,4,8] mid12 dec[2,2,2,2] (29.16M), rgb/B2 PSF, bs16/GPU 256x256, "
                      "L1 + 0.05*SSIM + 0.1*Phys_srgb, clip 0.01 + AdamW"),
    "cfg3": dict(batch=8, img=512, w=dict(w_l1=1.0, w_ssim=0.05, w_phys=0.1, w_perc=0.02, w_lpips=0.05, w_deltaE=0.02),
                 desc="cfg3: cfg2 model, rgb/B2 PSF, bs8/GPU 512x512, L1 + 0.05*SSIM + 0.1*Phys_srgb + 0.02*VGG19 perc "
                      "+ 0.05*LPIPS(vgg) + 0.02*DeltaE00, clip 0.01 + AdamW (synthetic VGG/LPIPS weights)"),
}
BATCH, IMG = 16, 256
W_L1, W_SSIM, W_PHYS = 1.0, 0.05, 0.1
FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 matrix/vector peak
BF16_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA peak
HBM_PEAK_GBPS = 8000.0


def nafblock_bytes(net, B, H, W):
    tot = 0
    h, w = H, W
    for i, n in enumerate(net.enc_blk_nums):
        tot += n * B * net.enc_chans[i] * h * w
        h, w = h // 2, w // 2
    tot += net.middle_blk_num * B * net.mid_chan * h * w
    for i, n in enumerate(net.dec_blk_nums):
        h, w = h * 2, w * 2
        tot += n * B * net.dec_chans[i] * h * w
    return 5 * tot * 4


def _pmc_traffic(cls):
    """HBM bytes per launch of a kernel class from the newest committed PMC record (profiles/*pmc_traffic.json,
    scripts/pmc_pass.sh + scripts/pmc_traffic.py: separate FETCH_SIZE / WRITE_SIZE passes, FETCH_SIZE doubled)."""
    import glob
    import re
    # newest record by version number (natural order: r01_v10 after r01_v9)
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_traffic.json")),
                   key=lambda f: [int(t) for t in re.findall(r"\d+", os.path.basename(f))])
    if not files:
        return None, None
    rec = json.load(open(files[-1])).get("classes", {}).get(cls)
    if rec is None:
        return None, None
    return round(rec["traffic_bytes_per_launch"]), os.path.relpath(files[-1], ROOT)


def cpu_baseline(state_dict, B=2, steps=2):
    """Time the oracle's training step (oracle/train_step.py, torch CPU fp32) on a bounded sample."""
    from oracle.train_step import OracleTrainer
    threads = min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16")), 16)
    torch.set_num_threads(threads)
    P = {k: v.detach().cpu() for k, v in state_dict.items()}
    ora = OracleTrainer(P, dict(enc_blk_nums=CFG["enc_blk_nums"], middle_blk_num=CFG["middle_blk_num"],
                                dec_blk_nums=CFG["dec_blk_nums"]), w_l1=W_L1, w_ssim=W_SSIM, w_phys=W_PHYS)
    g = torch.Generator().manual_seed(123)
    lq = torch.rand(B, 3, IMG, IMG, generator=g)
    gt = torch.rand(B, 3, IMG, IMG, generator=g)
    r = torch.ones(B, 1, 1, 1)
    ora.step(lq, gt, lq.clamp(0, 1), r)  # warm-up
    t0 = time.perf_counter()
    for _ in range(steps):
        ora.step(lq, gt, lq.clamp(0, 1), r)
    dt = (time.perf_counter() - t0) / steps
    return {"value": round(B / dt, 4), "unit": "img/s", "cores": threads, "kind": "port",
            "sample": f"oracle train step (torch CPU fp32), cfg2 model, bs={B} {IMG}x{IMG}, {steps} timed steps "
                      f"after 1 warm-up, {dt:.2f} s/step"}


def psnr_vs_cpu(net, dev):
    from oracle.nafnet import nafnet as oracle_nafnet
    g = torch.Generator().manual_seed(321)
    x = torch.rand(1, 3, IMG, IMG, generator=g)
    with torch.no_grad():
        y = net(x.to(dev)).cpu()
        P = {k: v.cpu() for k, v in net.state_dict().items()}
        yr = oracle_nafnet(P, x, CFG["enc_blk_nums"], CFG["middle_blk_num"], CFG["dec_blk_nums"])
    mse = ((y.double() - yr.double()) ** 2).mean().item()
    psnr = float("inf") if mse <= 1e-30 else 10 * torch.log10(torch.tensor(1.0 / mse)).item()
    return psnr, (y - yr).abs().max().item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--eager", action="store_true", help="time eager launches instead of HIP-graph replays")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp16", "fp32"],
                    help="bf16: bf16 MFMA operands + fp32 accumulation (the reference's AMP training); "
                         "fp32: fp32 everywhere (parity mode)")
    ap.add_argument("--workload", default="cfg2", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=0, help="per-GPU batch override (diagnostics; 0 = the workload's)")
    args = ap.parse_args()
    global BATCH, IMG
    wl = WORKLOADS[args.workload]
    BATCH, IMG = (args.batch or wl["batch"]), wl["img"]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from lowlight_image_enhancement_amd import _lib
    from lowlight_image_enhancement_amd.NewBP_model.newbp_net_arch import create_newbp_net
    from lowlight_image_enhancement_amd.train import NBPTrainer

    torch.manual_seed(0)
    net = create_newbp_net(in_channels=3, kernel_type="rgb", kernel_spec="B2", **CFG)
    init_sd = {k: v.clone() for k, v in net.state_dict().items()}
    net = net.to(dev)
    net.precision = args.precision
    tr = NBPTrainer(net, psf_mode="rgb", psf_spec="B2", **wl["w"])
    g = torch.Generator(device=dev).manual_seed(0 + rank)
    lq = torch.rand(BATCH, 3, IMG, IMG, device=dev, generator=g)
    gt = torch.rand(BATCH, 3, IMG, IMG, device=dev, generator=g)
    ratio = torch.ones(BATCH, 1, 1, 1, device=dev)
    short = (lq * ratio).clamp(0, 1)

    for _ in range(args.warmup):
        tr.step(lq, gt, short, ratio)
    logs_warm = tr.logs()

    # live per-kernel timing (HIP events on the launch stream) for the timed steps; each record carries the
    # launch's algorithmic flops and HBM bytes (operands read once, outputs written once)
    def mk(name, fl):
        def cb(a, e0, e1):
            prof[name].append((*fl(a), e0, e1))
        return cb

    def gemm_bf16_cost(a):  # (A,lda,amode,ascale,rows,adt,Bw,ldb,C,ldc,cmode,cdt,M,N,K,gh,gw,cs,bias,R,rscale,pre)
        M, N, K = a[12], a[13], a[14]
        ab, cb = (2 if a[5] else 4), (2 if a[11] else 4)
        by = M * K * ab + N * K * 2 + M * N * cb + (M * N * cb if a[19] is not None else 0) + \
            (M * N * 4 if a[21] is not None else 0)
        return 2.0 * M * N * K, by

    def gemm_f32_cost(a):  # (A,lda,amode,ascale,rows,B,ldb,bnk,C,ldc,cmode,M,N,K,gh,gw,cs,bias,R,rscale,pre)
        M, N, K = a[11], a[12], a[13]
        by = 4 * (M * K + N * K + M * N + (M * N if a[18] is not None else 0) + (M * N if a[20] is not None else 0))
        return 2.0 * M * N * K, by

    def wgrad_cost(a):  # (G,ldg,gm,X,ldx,xm,xs,rows,M,N,K,...,dtype)
        M, N, K = a[8], a[9], a[10]
        eb = 2 if a[-1] == 1 else 4
        return 2.0 * M * N * K, M * (N + K) * eb + N * K * 4

    def conv3x3_cost(a):  # (x,B,H,W,Cin,w,Cout,bias,mode,R,y,y_dtype): VGG implicit-GEMM conv, K = 9*Cin
        M, N, K = a[1] * a[2] * a[3], a[6], 9 * a[4]
        by = M * a[4] * 2 + N * K * 2 + M * N * (2 if a[11] else 4) + (M * N * 2 if a[9] is not None else 0)
        return 2.0 * M * N * K, by

    gemm_name = "gemm_f32" if args.precision == "fp32" else "gemm_bf16"
    prof = {gemm_name: [], "wgrad_f32": [], "conv3x3_bf16": []}
    _lib.PROFILE["conv3x3_bf16"] = mk("conv3x3_bf16", conv3x3_cost)
    _lib.PROFILE[gemm_name] = mk(gemm_name, gemm_f32_cost if args.precision == "fp32" else gemm_bf16_cost)
    _lib.PROFILE["wgrad_f32"] = mk("wgrad_f32", wgrad_cost)
    blk_events = []
    orig_fwd, orig_bwd = net._block_fwd, net._block_bwd

    def timed(fn, kind):
        def w(*a, **k):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            r = fn(*a, **k)
            e1.record()
            geo = (a[3], a[4], a[5], a[6]) if kind == "fwd" else a[4]  # (B, h, w, c)
            blk_events.append((e0, e1, kind, f"{geo[1]}x{geo[2]}xC{geo[3]}"))
            return r
        return w

    net._block_fwd, net._block_bwd = timed(orig_fwd, "fwd"), timed(orig_bwd, "bwd")

    # profiled pass: K eager steps with per-kernel HIP events on the launch stream (graph replays cannot carry them)
    step_events = []
    for _ in range(args.steps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        tr.step(lq, gt, short, ratio)
        e1.record()
        step_events.append((e0, e1))
    torch.cuda.synchronize()
    _lib.PROFILE.clear()
    net._block_fwd, net._block_bwd = orig_fwd, orig_bwd

    use_graph = world == 1 and not args.eager
    run = tr.graph_step if use_graph else tr.step
    if use_graph:
        run(lq, gt, short, ratio)  # capture + one replay, untimed
        run(lq, gt, short, ratio)

    # timed region: exactly K steps between barriers + device syncs
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run(lq, gt, short, ratio)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    logs = tr.logs()

    classes = {}
    for name, recs in prof.items():
        if not recs:
            continue
        ms = sum(e0.elapsed_time(e1) for _, _, e0, e1 in recs)
        classes[name] = (ms, sum(r[0] for r in recs), sum(r[1] for r in recs), len(recs))
    dom = max(classes, key=lambda k: classes[k][0])
    ms, fl, by, nl = classes[dom]
    peak_tf = FP32_PEAK_TFLOPS if args.precision == "fp32" else BF16_PEAK_TFLOPS
    tflops = fl / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
    gbps = by / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    # the binding roof is the one the kernel class is closer to (arithmetic intensity vs the ridge point)
    if fl / max(by, 1) < peak_tf * 1e12 / (HBM_PEAK_GBPS * 1e9):
        roof = {"bound": "hbm", "achieved": round(gbps, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(gbps / HBM_PEAK_GBPS, 4)}
    else:
        roof = {"bound": "mfma", "achieved": round(tflops, 3), "peak": peak_tf, "unit": "TFLOP/s",
                "frac": round(tflops / peak_tf, 4)}
    traffic, tsrc = _pmc_traffic(dom)
    roof.update({"traffic": traffic, "traffic_source": tsrc, "kernel": dom, "launches_per_step": nl // args.steps,
                 "ms_per_step": round(ms / args.steps, 3), "algorithmic_bytes_per_launch": round(by / max(nl, 1)),
                 "flop_intensity": round(fl / max(by, 1), 2), "tflops": round(tflops, 2),
                 "classes_ms_per_step": {k: round(v[0] / args.steps, 3) for k, v in classes.items()}})
    blk_ms = sum(e0.elapsed_time(e1) for e0, e1, _, _ in blk_events) / args.steps
    eager_step_ms = sum(e0.elapsed_time(e1) for e0, e1 in step_events) / args.steps
    per_level = {}
    for e0, e1, kind, lvl in blk_events:
        d = per_level.setdefault(lvl, {"blocks_fwd": 0, "fwd_ms": 0.0, "bwd_ms": 0.0})
        d[kind + "_ms"] += e0.elapsed_time(e1) / args.steps
        if kind == "fwd":
            d["blocks_fwd"] += 1
    for d in per_level.values():
        d["blocks_fwd"] //= args.steps
        d["fwd_ms"], d["bwd_ms"] = round(d["fwd_ms"], 3), round(d["bwd_ms"], 3)
    blk_bytes = nafblock_bytes(net, BATCH, IMG, IMG)
    # The eager per-block events include host-dispatch stalls at the small levels (the GPU outruns the launches
    # there); the NAFBlock GPU time is the timed step minus the non-NAFBlock part of the eager step (boundary convs,
    # down/up, loss head, optimizer: few large kernels, not dispatch-bound).
    step_ms_timed = elapsed / args.steps * 1e3
    nonblock_ms = max(eager_step_ms - blk_ms, 0.0)
    blk_ms_gpu = max(step_ms_timed - nonblock_ms, 1e-6)
    blk_gbps = blk_bytes / (blk_ms_gpu * 1e-3) / 1e9

    if rank == 0:
        step_ms = elapsed / args.steps * 1e3
        res = {
            "metric": METRIC if args.workload == "cfg2" else f"training images/sec ({args.workload})",
            "value": round(BATCH * world * args.steps / elapsed, 3),
            "unit": "img/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(step_ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": {"bf16": "bf16", "fp16": "f16", "fp32": "f32"}[args.precision],
            "data": "synthetic (U[0,1) sRGB, expo_ratio 1, torch default init, seed 0+rank)",
            "config": {"workload": wl["desc"],
                       "global_batch": BATCH * world, "image": IMG, "parallelism": f"dp{world}",
                       "launch": "hip-graph replay" if use_graph else "eager"},
            "roofline": roof,
            "nafblock_roofline": {"bytes_per_step": blk_bytes, "ms_per_step": round(blk_ms_gpu, 3),
                                  "ms_method": "timed step - non-NAFBlock part of the eager step",
                                  "eager_blocks_ms_per_step": round(blk_ms, 3),
                                  "per_level_eager": per_level,
                                  "achieved_GBps": round(blk_gbps, 1), "peak_GBps": HBM_PEAK_GBPS,
                                  "frac": round(blk_gbps / HBM_PEAK_GBPS, 4)},
            "losses": logs,
        }
        if world == 1:
            psnr, maxabs = psnr_vs_cpu(net, dev)
            res["psnr_vs_cpu_ref_db"] = round(psnr, 2) if psnr != float("inf") else "inf"
            res["max_abs_vs_cpu_ref"] = maxabs
            if not args.no_cpu_baseline and args.workload == "cfg2":
                res["cpu_baseline"] = cpu_baseline(init_sd)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
