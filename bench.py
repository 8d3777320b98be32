"""Benchmark: training images/sec of the NewBP-NAFNet hot path on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1], the 1-GPU headline config): NAFNet width 32, enc [2,2,4,8], middle 12,
dec [2,2,2,2] (29.16 M params), rgb/B2 crosstalk PSF, 16 x 3 x 256 x 256 synthetic sRGB per GPU,
HybridLoss terms L1 + SSIM + Phys_srgb, global-norm clip 0.01 + AdamW.  One "step" = forward + loss + backward
(+ bucketed RCCL all-reduce when N > 1) + clip + AdamW, all HIP kernels.  Default precision fp16 (fp16 storage and
MFMA operands, fp32 accumulation / statistics / parameters, dynamic loss scaling): the reference's AMP dtype.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--precision fp16|bf16|fp32] [--workload cfg2|cfg3|cfg4] [--quick]

N > 1 runs one process per GPU.  Either under a launcher (python -m torch.distributed.run --nproc-per-node N
--master-addr 127.0.0.1 bench.py --gpus N ...: WORLD_SIZE must equal N, else the bench exits non-zero), or stand-alone
(`python bench.py --gpus N` with WORLD_SIZE unset): the bench then starts N local ranks itself, torchrun-style
(RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT in each child's environment; the DDP launch
contract of NAFNet_base/basicsr/train.py:54-63, utils/dist_util.py:28-40), before anything touches the GPU, and exits
with the first failing rank's status.  Fewer visible GPUs than N is an error (NBP_BENCH_REHEARSE=1 excepted: every
rank on cuda:0 over gloo, a rehearsal of the N > 1 path on a one-GPU box, tagged in the JSON line).

Rank 0 prints ONE JSON line.
* `roofline`: the dominant kernel class (by measured time among the classes below), timed live with HIP events on
  the launch stream over K eager steps; achieved = its algorithmic bytes (or FLOPs) per launch / its average launch
  duration.  Classes: `gemm16` (every 16-bit MFMA GEMM entry: nbp_gemm_bf16 + the fused-epilogue entries
  nbp_gemm_res_ln / nbp_dgrad_ln_bwd / nbp_dgrad_sg_rc), `wgrad`, `dw_bwd` (nbp_sca_sg_dw_bwd), `dw_fwd`
  (nbp_dw_sg_pool_fwd); rocprof kernel names in ROCPROF_KERNELS.
* `nafblock_roofline`: the north-star figure, NAFBlock fwd+bwd algorithmic bytes (5*B*C*H*W*s per block,
  s = the storage bytes per element of this precision) vs 8 TB/s.
* `modes` / `cfg3` / `cfg4` (rank 0, N = 1, unless --quick): the other precision modes on the same workload, a bounded
  BASELINE configs[2] sample (bs 8 x 512^2, all six HybridLossPlus terms, synthetic VGG / LPIPS weights), and the
  configs[3] model (w64, bs 16 per GPU: the scaling config; `--workload cfg4` times it at any N).
* `cpu_baseline`: the CPU oracle (oracle/, kind "port") at the full cfg2 batch on this box's host cores (median of 3
  timed steps after 1 warm-up), as BASELINE.md prescribes.
* `psnr_vs_cpu_ref_db`: GPU vs CPU-oracle output on the same weights and input, at the reference's init (zero layer
  scales: every block an identity) and with active blocks (beta, gamma ~ N(0, 0.2), `psnr_active_blocks_db`).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "training images/sec at 256×256 bs=16 (1/2/4/8 GPU) + PSNR vs CPU ref"
CFG = dict(width=32, enc_blk_nums=[2, 2, 4, 8], middle_blk_num=12, dec_blk_nums=[2, 2, 2, 2])
BLK = {k: v for k, v in CFG.items() if k != "width"}
# BASELINE.json configs[1] (the headline) and configs[2] (VGG19 perceptual + LPIPS(alex) + ΔE00, bs8 512² as
# BASELINE.json names it; weights from configs/colab/sid_newbp_rgb.yml:78-96; synthetic offline VGG / AlexNet weights)
CFG4 = dict(CFG, width=64)
WORKLOADS = {
    "cfg2": dict(batch=16, img=256, w=dict(w_l1=1.0, w_ssim=0.05, w_phys=0.1),
                 desc="cfg2: NAFNet w32 enc[2,2,4,8] mid12 dec[2,2,2,2] (29.16M), rgb/B2 PSF, bs16/GPU 256x256, "
                      "L1 + 0.05*SSIM + 0.1*Phys_srgb, clip 0.01 + AdamW"),
    "cfg3": dict(batch=8, img=512, w=dict(w_l1=1.0, w_ssim=0.05, w_phys=0.1, w_perc=0.02, w_lpips=0.05, w_deltaE=0.02,
                                          lpips_net="alex"),
                 desc="cfg3: cfg2 model, rgb/B2 PSF, bs8/GPU 512x512, L1 + 0.05*SSIM + 0.1*Phys_srgb + 0.02*VGG19 perc "
                      "+ 0.05*LPIPS(alex) + 0.02*DeltaE00, clip 0.01 + AdamW (synthetic VGG/LPIPS weights)"),
    # BASELINE.json configs[3], the >= 6.5x scaling config: w64 (115.98M), bs 16 per GPU (128 global on 8), the
    # stressed R > G > B PSF family (S2; the reference only describes it, newbp_layer.py here defines it)
    "cfg4": dict(batch=16, img=256, w=dict(w_l1=1.0, w_ssim=0.05, w_phys=0.1), model=CFG4, psf="S2",
                 desc="cfg4: NAFNet w64 enc[2,2,4,8] mid12 dec[2,2,2,2] (115.98M), rgb/S2 stressed PSF (R>G>B), "
                      "bs16/GPU 256x256, L1 + 0.05*SSIM + 0.1*Phys_srgb, clip 0.01 + AdamW"),
    # BASELINE.json configs[4], the RAW / linear-domain path: 4 x MI355X bs 32 at 1024^2 = 8 images per GPU, fp16
    # compute; phys_cons_raw (metrics/phys_consistency.py:260-320) with expo_ratio in {100, 250, 300} and fp32
    # accumulation evaluated on each step's output
    "cfg5": dict(batch=8, img=1024, w=dict(w_l1=1.0, w_ssim=0.05, w_phys=0.1), raw_ratios=(100.0, 250.0, 300.0),
                 desc="cfg5: cfg2 model, rgb/B2 PSF, bs8/GPU 1024x1024, L1 + 0.05*SSIM + 0.1*Phys_srgb, clip 0.01 + "
                      "AdamW; phys_cons_raw(out, short, psf, expo_ratio in {100,250,300}) on the fp16-cast output "
                      "(fp32 accumulation)"),
}
FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 matrix/vector peak
MFMA16_PEAK_TFLOPS = 2500.0  # dense bf16 / fp16 MFMA peak
HBM_PEAK_GBPS = 8000.0
ESIZE = {"fp32": 4, "bf16": 2, "fp16": 2}
ROCPROF_KERNELS = {"gemm16": ["gemm_glds_kernel", "gemm_bf16_kernel", "gemm_skinny_kernel"], "gemm_f32": ["gemm_f32_kernel"],
                   "wgrad_narrow": ["wgrad_bf16_kernel", "wgrad_f32_kernel", "wgrad_narrow_full"], "wgrad_group": ["wgrad_bf16_wide_group"],
                   "reduce": ["reduce_multi_kernel", "reduce_table_kernel", "layer_scale_grad_kernel"],
                   "dw_bwd": ["dw_bwd_tiled"], "dw_fwd": ["dw_sg_pool_tiled"], "c1dw": ["c1_dw_sg_pool_img"],
                   "c1dw_tile_fwd": ["c1dw_fwd_tile"], "c1dw_tile_bwd": ["c1dw_bwd_tile"]}
# ONE-kernel classes (one template instance each), timed per launch inside the library (nbp_launch_timing: events
# around that launch alone on its stream) and keyed by the instance name the library records; the headline `roofline`
# is the one with the most time per step (the dominant kernel).  Their rocprof names, as regexes over the mangled
# names of kernel_stats.csv (exactly one instance per regex and dtype: tests/test_bench_launch.py checks the committed
# record).
INSTANCES = {"c1dw_bwd_tile<T,32>": "c1dw_bwd_L0", "c1dw_bwd_tile<T,64>": "c1dw_bwd_L1",
             "c1dw_bwd_tile<T,32,sca>": "c1dw_bwd_sca_L0", "c1dw_bwd_tile<T,64,sca>": "c1dw_bwd_sca_L1",
             "dw_bwd_tiled<T,true,32>": "dw_bwd_32", "dw_bwd_tiled<T,true,16>": "dw_bwd_16",
             "dw_bwd_tiled<T,true,32,sca>": "dw_bwd_sca_32", "dw_bwd_tiled<T,true,16,sca>": "dw_bwd_sca_16",
             "wgrad_bf16_wide_group<3,512,2>": "wgrad_group_512", "wgrad_bf16_wide_group<3,768,4>": "wgrad_group_768",
             "reduce_multi_kernel": "reduce_multi", "reduce_table_kernel": "reduce_table",
             "layer_scale_grad_kernel": "layer_scale_grad",
             "ffn_rows_fwd<512>": "ffn_rows_512", "ffn_rows_fwd<256>": "ffn_rows_256", "ffn_rows_fwd<128>": "ffn_rows_128",
             "ffn_rows_bwd<512>": "ffn_rows_bwd_512", "ffn_rows_bwd<256>": "ffn_rows_bwd_256",
             "ffn_rows_bwd<128>": "ffn_rows_bwd_128", "ffn_rows_bwd<512,pre>": "ffn_rows_bwd_pre_512",
             "ffn_rows_bwd<256,pre>": "ffn_rows_bwd_pre_256", "ffn_rows_bwd<128,pre>": "ffn_rows_bwd_pre_128"}
SINGLE_KERNEL = tuple(INSTANCES.values())
ROCPROF_KERNELS.update({
    "c1dw_bwd_L0": [r"c1dw_bwd_tileI{T}Li32ELi\d+ELb[01]E(Lb0E)?E"],
    "c1dw_bwd_L1": [r"c1dw_bwd_tileI{T}Li64ELi\d+ELb[01]E(Lb0E)?E"],
    "c1dw_bwd_sca_L0": [r"c1dw_bwd_tileI{T}Li32ELi\d+ELb[01]ELb1EE"],
    "c1dw_bwd_sca_L1": [r"c1dw_bwd_tileI{T}Li64ELi\d+ELb[01]ELb1EE"],
    "dw_bwd_32": [r"dw_bwd_tiledI{T}Lb1ELi32E(Lb0E)?E"], "dw_bwd_16": [r"dw_bwd_tiledI{T}Lb1ELi16E(Lb0E)?E"],
    "dw_bwd_sca_32": [r"dw_bwd_tiledI{T}Lb1ELi32ELb1EE"], "dw_bwd_sca_16": [r"dw_bwd_tiledI{T}Lb1ELi16ELb1EE"],
    "wgrad_group_512": [r"wgrad_bf16_wide_groupI{T}Li3ELi512ELi2EE"],
    "wgrad_group_768": [r"wgrad_bf16_wide_groupI{T}Li3ELi768ELi4EE"],
    "reduce_multi": [r"reduce_multi_kernel"], "reduce_table": [r"reduce_table_kernel"],
    "layer_scale_grad": [r"layer_scale_grad_kernel"],
    "ffn_rows_512": [r"ffn_rows_fwdI{T}Li512EE"], "ffn_rows_256": [r"ffn_rows_fwdI{T}Li256EE"],
    "ffn_rows_128": [r"ffn_rows_fwdI{T}Li128EE"], "ffn_rows": ["ffn_rows_fwd", "ffn_rows_bwd"],
    "ffn_rows_bwd_512": [r"ffn_rows_bwdI{T}Li512ELb0EE"], "ffn_rows_bwd_256": [r"ffn_rows_bwdI{T}Li256ELb0EE"],
    "ffn_rows_bwd_128": [r"ffn_rows_bwdI{T}Li128ELb0EE"], "ffn_rows_bwd_pre_512": [r"ffn_rows_bwdI{T}Li512ELb1EE"],
    "ffn_rows_bwd_pre_256": [r"ffn_rows_bwdI{T}Li256ELb1EE"], "ffn_rows_bwd_pre_128": [r"ffn_rows_bwdI{T}Li128ELb1EE"]})
# the Itanium mangling of the storage type in those names
MANGLED_T = {"fp16": "DF16_", "bf16": "DF16b", "fp32": "f"}
UNIT_DEF = {
    "dw_bwd_32": "SURVEY §8(d)-style per pixel: dh C + t2 2C + t1 2C read, dt1 2C written = 7*C*s bytes per pixel "
                 "(s = storage bytes), x B*H*W pixels of the launch (the 32-wide tile kernel at the levels that store "
                 "the tape: 2-3 at cfg2; levels 0-1 rebuild it in c1dw_bwd_tile)",
    "dw_bwd_16": "as dw_bwd_32 (7*C*s bytes per pixel), the 16-wide tile kernel (the 16 x 16 level)",
    "dw_bwd_sca_32": "as dw_bwd_32, + the SCA backward folded in: the channel-dot slab (B x chunks x C) and W_sca "
                     "(C^2) read, dW_sca (C^2) written, fp32",
    "dw_bwd_sca_16": "as dw_bwd_sca_32, the 16-wide tile kernel (the 16 x 16 level)",
    "wgrad_group_512": "per grouped launch of this instance (128-column tiles): each problem's operands read once, "
                       "M*(N+K)*s, + its fp32 dW (+db) written once; the split-M fp32 slabs it writes instead are the "
                       "wgrad_group class's `slab_bytes_per_step`",
    "wgrad_group_768": "as wgrad_group_512, the 256-column-tile instance (the 16 x 16 level's plain problems, unsplit)",
    "reduce_multi": "per reduce_multi_kernel launch: the fp32 slabs read once + the reduced outputs written once",
    "reduce_table": "per reduce_table_kernel launch (a whole flush from the device descriptor table): the fp32 slabs "
                    "read once + the reduced outputs written once",
    "layer_scale_grad": "per layer_scale_grad_kernel launch: U, V, W, b read, dW, db, dscale written (fp32)",
    "c1dw_bwd_L0": "per pixel: dh C + n1 C read, dt1 2C written = 4*C*s bytes (s = storage bytes; t1 / t2 rebuilt on "
                   "chip, never read), x B*H*W pixels of the launch (level 0: C 32 at 256^2), + the conv1 weight",
    "c1dw_bwd_L1": "as c1dw_bwd_L0 at level 1 (C 64 at 128^2)",
    "c1dw_bwd_sca_L0": "as c1dw_bwd_L0, + the SCA backward folded in: the channel-dot slab (B x chunks x C) and W_sca "
                       "(C^2) read, dW_sca (C^2) written, fp32",
    "c1dw_bwd_sca_L1": "as c1dw_bwd_sca_L0 at level 1 (C 64 at 128^2)",
    "ffn_rows_512": "per pixel: g C + x C read, y + n2 + t4 (2C) + g2 + out (+ the next n1) written = 8-9 C s bytes, "
                    "+ the three weights (4 C^2 s) once per launch (the middle level: C 512 at 16^2)",
    "ffn_rows_256": "as ffn_rows_512 at C 256 (32^2)", "ffn_rows_128": "as ffn_rows_512 at C 128 (64^2)",
    "ffn_rows_bwd_512": "per pixel: dout C + t4 2C + y C + g C read, dt4 2C + dy C + dh C written = 9 C s bytes, + the "
                        "three weights (4 C^2 s) once per launch and the per-32-row partial sums (the middle level)",
    "ffn_rows_bwd_256": "as ffn_rows_bwd_512 at C 256 (32^2)", "ffn_rows_bwd_128": "as ffn_rows_bwd_512 at C 128 (64^2)",
    "ffn_rows_bwd_pre_512": "as ffn_rows_bwd_512 (dout made in-kernel, not read), + the following block's conv1 input "
                            "gradient: dt1 2C + x C + dres C read, dx C written = 14 C s bytes per pixel, + four "
                            "weights (6 C^2 s) once per launch",
    "ffn_rows_bwd_pre_256": "as ffn_rows_bwd_pre_512 at C 256 (32^2)",
    "ffn_rows_bwd_pre_128": "as ffn_rows_bwd_pre_512 at C 128 (64^2)",
}


def nafblock_bytes(net, B, H, W, esize):
    tot = 0
    h, w = H, W
    for i, n in enumerate(net.enc_blk_nums):
        tot += n * B * net.enc_chans[i] * h * w
        h, w = h // 2, w // 2
    tot += net.middle_blk_num * B * net.mid_chan * h * w
    for i, n in enumerate(net.dec_blk_nums):
        h, w = h * 2, w * 2
        tot += n * B * net.dec_chans[i] * h * w
    return 5 * tot * esize


# ------------------------------------------------------------------ algorithmic work per launch, by C-ABI entry
def _e(dt):
    return 4 if dt == 0 else 2


def cost_gemm16(a):  # (A,lda,amode,ascale,rows,adt,Bw,ldb,C,ldc,cmode,cdt,M,N,K,gh,gw,cs,bias,R,rscale,pre)
    M, N, K, cm = a[12], a[13], a[14], a[10]
    ea, ec = _e(a[5]), _e(a[11])
    by = M * K * ea + N * K * 2
    if cm == 5:  # SimpleGate backward: dt [M][2N] out, t [M][2N] in
        by += 4 * M * N * ec
    elif cm == 4:  # SimpleGate forward: t [M][N] (unless dropped) + g [M][N/2]
        by += (M * N * ec if a[8] is not None else 0) + M * N // 2 * ec
    else:
        by += M * N * ec + (M * N * ec if a[19] is not None else 0) + (M * N * ec if a[21] is not None and cm != 8 else 0)
    return 2.0 * M * N * K, by


def cost_res_ln(a):  # (A,lda,amode,ascale,rows,Bw,ldb,C,M,N,K,bias,R,rscale,lnw,lnb,nout,stats,eps,dt)
    M, N, K = a[8], a[9], a[10]
    return 2.0 * M * N * K, (M * K + N * K + 3 * M * N) * 2 + 8 * M


def cost_dgrad_ln(a):  # (A,lda,Wt,ldb,M,N,K,x,stats,lnw,dres,dx,dlnw,dlnb,ws,n_ws,dt)
    M, N, K = a[4], a[5], a[6]
    return 2.0 * M * N * K, (M * K + N * K + 3 * M * N) * 2 + 8 * M


def cost_sg_rc(a):  # (A,lda,Wt,ldb,A2,W2,b2,C,M,N,K,dt): dgrad + the rebuilt conv4 forward
    M, N, K = a[8], a[9], a[10]
    return 2.0 * M * N * K + 4.0 * M * N * K, (2 * M * K + 3 * N * K + 2 * M * N) * 2


def cost_wgrad(a):  # (G,ldg,gm,X,ldx,xm,xs,rows,M,N,K,gh,gw,csg,csx,dW,db,ws,n_ws,dtype): operands once + fp32 dW/db
    M, N, K = a[8], a[9], a[10]
    return 2.0 * M * N * K, M * (N + K) * _e(a[-1]) + N * K * 4 + (N * 4 if a[16] is not None else 0)


def cost_dw_bwd(a):  # (dh,a,ds,t2,t1,wdw,dt1,dwdw,dbdw,ws,B,h,w,c,dt): dh C + t2 2C + t1 2C in, dt1 2C out
    M, c = a[10] * a[11] * a[12], a[13]
    return 2.0 * M * 2 * c * 18, 7 * M * c * _e(a[14])


def cost_sca_dw_bwd(a):  # (dh,a,da_slab,chunks,wsca,mean,dwsca,dbsca,t2,t1,wdw,dt1,dwdw,dbdw,ws,B,h,w,c,dt): as
    # cost_dw_bwd + the SCA backward: the channel-dot slab and W_sca read, dW_sca written (fp32)
    B, c = a[15], a[18]
    M = B * a[16] * a[17]
    return (2.0 * M * 2 * c * 18 + 4.0 * B * c * c, 7 * M * c * _e(a[19]) + 4 * (B * a[3] * c + 2 * c * c))


def cost_dw_fwd(a):  # (t1,w,b,t2,g,pool,B,h,w,c,dt): t1 2C in, t2 2C + g C out
    M, c = a[6] * a[7] * a[8], a[9]
    return 2.0 * M * 2 * c * 9, (2 + (2 if a[3] is not None else 0) + 1) * M * c * _e(a[10])


def cost_ffn(a):  # (n2,W4,b4,W5,b5,y,gamma,lnw,lnb,out,nout,stats,M,C,eps,dt): n2 + y in, out (+ nout + stats) out
    M, C = a[12], a[13]
    by = (3 * M * C + 3 * C * C + (M * C if a[10] is not None else 0)) * 2 + (8 * M if a[11] is not None else 0)
    return 2.0 * M * 2 * C * C + 2.0 * M * C * C, by


def cost_sg_rc_wg(a):  # cost_sg_rc + the folded weight gradients U = dout^T g, dW4 = dt4^T n2 (fp32 partial slabs)
    fl, by = cost_sg_rc(a)
    M, N, K = a[8], a[9], a[10]
    return fl + 2.0 * M * N * N + 2.0 * M * 2 * N * K, by


def cost_dgrad_ln_wg(a):  # cost_dgrad_ln + the folded conv1 weight gradient dW1 = dt1^T n1 (n1 rebuilt, not read)
    fl, by = cost_dgrad_ln(a)
    M, N, K = a[4], a[5], a[6]
    return fl + 2.0 * M * N * K, by


def cost_c1dw(a):  # (n1,w1,b1,wdw,bdw,t1,t2,g,pool,B,h,w,c,dt): n1 C in, t1 2C (+ t2 2C) + g C out, conv1 weight
    M, c = a[9] * a[10] * a[11], a[12]
    by = (M * c + 2 * M * c + (2 * M * c if a[6] is not None else 0) + M * c + 2 * c * c) * _e(a[13])
    return 2.0 * M * 2 * c * c + 2.0 * M * 2 * c * 9, by


def cost_c1dw_fwd_tile(a):  # (n1,w1,b1,wdw,bdw,t1,t2,g,pool,B,h,w,c,dt): n1 C in, g C out (+ t1 / t2 2C when kept)
    M, c = a[9] * a[10] * a[11], a[12]
    by = (2 * M * c + (2 * M * c if a[5] is not None else 0) + (2 * M * c if a[6] is not None else 0) + 2 * c * c) * _e(a[13])
    return 2.0 * M * 2 * c * c + 2.0 * M * 2 * c * 9, by


def cost_sca_c1dw_bwd_tile(a):  # (dh,a,da_slab,chunks,wsca,mean,dwsca,dbsca,n1,w1,b1,wdw,bdw,dt1,dwdw,dbdw,ws,B,h,w,c,
    # dt): cost_c1dw_bwd_tile + the folded SCA backward (the channel-dot slab and W_sca read, dW_sca written, fp32)
    B, c = a[17], a[20]
    M = B * a[18] * a[19]
    return (2.0 * M * 2 * c * c + 3 * 2.0 * M * 2 * c * 9 + 4.0 * B * c * c,
            (4 * M * c + 2 * c * c) * _e(a[21]) + 4 * (B * a[3] * c + 2 * c * c))


def cost_c1dw_bwd_tile(a):  # (dh,a,ds,n1,w1,b1,wdw,bdw,dt1,dwdw,dbdw,ws,B,h,w,c,dt): dh C + n1 C in, dt1 2C out
    M, c = a[12] * a[13] * a[14], a[15]
    return 2.0 * M * 2 * c * c + 3 * 2.0 * M * 2 * c * 9, (4 * M * c + 2 * c * c) * _e(a[16])




def cost_ffn_rows(a):  # (g,a,hw,x,w3,b3,beta,lnw2,lnb2,w4,b4,w5,b5,gamma,lnw1,lnb1,y,n2,st2,t4,g2,out,nn1,nst1,M,C,eps,dt)
    M, C = a[24], a[25]
    nxt = a[14] is not None
    return 8.0 * M * C * C, (M * C * (9 if nxt else 8) + 4 * C * C) * 2 + M * 8 * (2 if nxt else 1)


def cost_ffn_rows_bwd(a):  # (dout,t4,y,st2,lnw2,g,w5t,w4t,w3t,dt4,dy,dh,sw,sb,da,dt1,w1t,x1,st1,lnw1,dres1,dx1,sw1,sb1,M,C,hw,dt)
    M, C = a[24], a[25]
    pre = a[15] is not None  # + the following block's conv1 input gradient / norm1 backward
    return (8.0 + 4.0 * pre) * M * C * C, ((M * C * (14 if pre else 9) + (6 if pre else 4) * C * C) * 2
                                           + M * 8 * (2 if pre else 1) + (5 if pre else 3) * (M // 32) * C * 4)


def cost_gemm_f32(a):  # (A,lda,amode,ascale,rows,B,ldb,bnk,C,ldc,cmode,M,N,K,gh,gw,cs,bias,R,rscale,pre)
    M, N, K = a[11], a[12], a[13]
    return 2.0 * M * N * K, 4 * (M * K + N * K + M * N + (M * N if a[18] is not None else 0))


def rec_plain(cls, cost):
    """one C-ABI call = one kernel launch of `cls`"""
    return lambda a: [(cls, *cost(a), 1, 0.0)]


def rec_wgrad(a):
    """nbp_wgrad_f32: a wide problem inside an open level group is only queued (no GPU work: not a launch of its
    own; its bytes are counted in the group launch), the others launch one wgrad kernel writing S fp32 slabs."""
    st = _lib_stats(0)
    if st[0]:
        return []
    fl, by = cost_wgrad(a)
    return [("wgrad_narrow", fl, by, 1, st[2])]


def rec_wgroup(a):
    """nbp_wgrad_group(0): the level's grouped launch(es): operands read once + fp32 dW / db written once per problem
    (algorithmic); the fp32 split-M slabs the launch writes instead are reported as slab bytes (the reduce class
    reads them back)."""
    if a[0]:
        return []
    st = _lib_stats(2)
    if not st[5]:
        return []
    return [("wgrad_group", st[1], st[2] + st[3], int(st[5]), st[4])]


def rec_flush(a):
    """nbp_grad_reduce_flush: the stage's deferred slab reductions (+ layer-scale post-ops): fp32 slabs read once,
    outputs written once, per reduce_multi_kernel launch."""
    st = _lib_stats(1)
    if not st[3]:
        return []
    return [("reduce", 0.0, st[1] + st[2], int(st[3]), 0.0)]


def _lib_stats(which):
    from lowlight_image_enhancement_amd import _lib
    return _lib.last_call_stats(which)


# C-ABI entry -> records [(class, FLOPs, algorithmic bytes, kernel launches, fp32 slab bytes written)]
ENTRIES = {"gemm_bf16": rec_plain("gemm16", cost_gemm16), "gemm_res_ln": rec_plain("gemm16", cost_res_ln),
           "dgrad_ln_bwd": rec_plain("gemm16", cost_dgrad_ln), "dgrad_sg_rc": rec_plain("gemm16", cost_sg_rc),
           "gemm_f32": rec_plain("gemm_f32", cost_gemm_f32), "wgrad_f32": rec_wgrad, "wgrad_group": rec_wgroup,
           "grad_reduce_flush": rec_flush, "sca_sg_dw_bwd": rec_plain("dw_bwd", cost_dw_bwd),
           "sca_dw_bwd": rec_plain("dw_bwd", cost_sca_dw_bwd),
           "dw_sg_pool_fwd": rec_plain("dw_fwd", cost_dw_fwd), "gemm_ffn": rec_plain("gemm16", cost_ffn),
           "dgrad_sg_rc_wg": rec_plain("gemm16", cost_sg_rc_wg),
           "dgrad_ln_bwd_wg": rec_plain("gemm16", cost_dgrad_ln_wg), "c1_dw_sg_pool": rec_plain("c1dw", cost_c1dw),
           "c1dw_fwd_tile": rec_plain("c1dw_tile_fwd", cost_c1dw_fwd_tile),
           "c1dw_bwd_tile": rec_plain("c1dw_tile_bwd", cost_c1dw_bwd_tile),
           "sca_c1dw_bwd_tile": rec_plain("c1dw_tile_bwd", cost_sca_c1dw_bwd_tile),
           "ffn_rows_fwd": rec_plain("ffn_rows", cost_ffn_rows), "ffn_rows_bwd": rec_plain("ffn_rows", cost_ffn_rows_bwd)}


def _pmc_newest_key(f):
    """Record order under profiles/: round number first, a round's "final" record after its numbered ones (r04_final >
    r04_v1)."""
    import re
    rel = os.path.relpath(f, os.path.join(ROOT, "profiles"))
    nums = [int(t) for t in re.findall(r"\d+", rel)]
    return (nums[:1], "final" in rel, nums)


def _pmc_traffic(cls):
    """HBM bytes per launch of a kernel class from the newest committed PMC record (profiles/[*/]*pmc_traffic.json,
    scripts/pmc_pass.sh + scripts/pmc_traffic.py: separate FETCH_SIZE / WRITE_SIZE passes, FETCH_SIZE doubled)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_traffic.json"))
                   + glob.glob(os.path.join(ROOT, "profiles", "*", "*pmc_traffic.json")), key=_pmc_newest_key)
    if not files:
        return None, None
    rec = json.load(open(files[-1])).get("classes", {}).get(cls)
    if rec is None:
        return None, os.path.relpath(files[-1], ROOT)
    return round(rec["traffic_bytes_per_launch"]), os.path.relpath(files[-1], ROOT)


def _class_line(cls, v, steps, peak_tf, mt):
    """One kernel class of the profiled pass, per KERNEL launch (the unit of the PMC traffic record) and per step:
    launches, average launch, algorithmic bytes / FLOPs, the fraction of the HBM and MFMA roofs they reach, the PMC
    traffic and its ratio to the algorithmic bytes, and the fp32 split-M slab bytes the class writes (read back by
    the `reduce` class)."""
    ms, fl, by, nl, ncall, slab = v
    gbps = by / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    tfl = fl / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
    traffic, _ = _pmc_traffic(cls)
    alg = by / max(nl, 1)
    line = {"rocprof_kernels": [r.format(T=mt) for r in ROCPROF_KERNELS[cls]], "ms_per_step": round(ms / steps, 3),
            "launches_per_step": round(nl / steps, 2), "c_abi_calls_per_step": round(ncall / steps, 2),
            "avg_launch_us": round(ms * 1e3 / max(nl, 1), 2), "algorithmic_bytes_per_launch": round(alg),
            "algorithmic_bytes_per_step": round(by / steps), "algorithmic_flops_per_launch": round(fl / max(nl, 1)),
            "GBps": round(gbps, 1), "hbm_frac": round(gbps / HBM_PEAK_GBPS, 4), "TFLOPs": round(tfl, 2),
            "mfma_frac": round(tfl / peak_tf, 4), "traffic": traffic,
            "traffic_per_step": None if traffic is None else round(traffic * nl / steps),
            "traffic_over_algorithmic": None if traffic is None or alg <= 0 else round(traffic / alg, 3)}
    if slab:
        line["slab_bytes_per_step"] = round(slab / steps)
    return line


def nproc() -> int:
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return min(n, int(omp)) if omp.isdigit() and int(omp) > 0 else n


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(state_dict, B=16, img=256, timed=3):
    """The oracle's training step (oracle/train_step.py, torch CPU fp32; pinned against the reference by the golden
    fixtures) at the full cfg2 batch: set_num_threads(nproc), 1 warm-up + `timed` steps, img/s = B / median step
    (BASELINE.md 'CPU-baseline plan').  nproc = the CPUs this process may run on, capped by OMP_NUM_THREADS (what
    coreutils nproc reports: the GPU box exports OMP_NUM_THREADS=16, its per-GPU CPU share)."""
    from oracle.train_step import OracleTrainer
    cores = nproc()
    torch.set_num_threads(cores)
    P = {k: v.detach().cpu() for k, v in state_dict.items()}
    ora = OracleTrainer(P, BLK, **WORKLOADS["cfg2"]["w"])
    g = torch.Generator().manual_seed(123)
    lq = torch.rand(B, 3, img, img, generator=g)
    gt = torch.rand(B, 3, img, img, generator=g)
    r = torch.ones(B, 1, 1, 1)
    ora.step(lq, gt, lq.clamp(0, 1), r)  # warm-up
    ts = []
    for i in range(timed):
        t0 = time.perf_counter()
        ora.step(lq, gt, lq.clamp(0, 1), r)
        ts.append(time.perf_counter() - t0)
        print(f"[bench] cpu baseline step {i + 1}/{timed}: {ts[-1]:.2f} s", file=sys.stderr, flush=True)
    med = statistics.median(ts)
    return {"value": round(B / med, 4), "unit": "img/s", "cores": cores, "kind": "port",
            "sample": f"oracle train step (torch {torch.__version__} CPU fp32: fwd + L1/SSIM/Phys_srgb + bwd + clip + "
                      f"AdamW), cfg2 model at the full bs={B} {img}x{img}, median of {timed} timed steps after 1 "
                      f"warm-up ({', '.join(f'{t:.2f}' for t in ts)} s), torch.set_num_threads({cores}) = nproc "
                      f"(os.cpu_count() {os.cpu_count()}); CPU {_cpu_model()}"}


def psnr_vs_cpu(net, dev, img, active=False):
    """GPU output vs the CPU oracle's on the same weights and input (1 image).  active: random layer scales."""
    from oracle.nafnet import nafnet as oracle_nafnet
    backup = None
    if active:
        backup = net.flat.data.clone()
        g = torch.Generator().manual_seed(7)
        with torch.no_grad():
            for k, e in net.entries.items():
                if k.endswith("beta") or k.endswith("gamma"):
                    net.flat.data[e.offset:e.offset + e.numel] = (0.2 * torch.randn(e.numel, generator=g)).to(dev)
    g = torch.Generator().manual_seed(321)
    x = torch.rand(1, 3, img, img, generator=g)
    with torch.no_grad():
        y = net(x.to(dev)).cpu()
        P = {k: v.cpu() for k, v in net.state_dict().items()}
        yr = oracle_nafnet(P, x, **BLK)
    if backup is not None:
        net.flat.data.copy_(backup)
    mse = ((y.double() - yr.double()) ** 2).mean().item()
    psnr = float("inf") if mse <= 1e-30 else 10 * torch.log10(torch.tensor(1.0 / mse)).item()
    return (round(psnr, 2) if psnr != float("inf") else "inf"), (y - yr).abs().max().item()


def make_trainer(dev, workload, precision, seed=0):
    from lowlight_image_enhancement_amd.NewBP_model.newbp_net_arch import create_newbp_net
    from lowlight_image_enhancement_amd.train import NBPTrainer
    wl = WORKLOADS[workload]
    spec = wl.get("psf", "B2")
    torch.manual_seed(seed)
    net = create_newbp_net(in_channels=3, kernel_type="rgb", kernel_spec=spec, **wl.get("model", CFG))
    init_sd = {k: v.clone() for k, v in net.state_dict().items()}
    net = net.to(dev)
    net.precision = precision
    tc = os.environ.get("NBP_C1DW_TILE_C")  # A/B experiments only: the levels (channel counts) on the tile path
    if tc is not None:
        net.c1dw_tile_channels = tuple(int(c) for c in tc.split(",") if c)
    if os.environ.get("NBP_LN_WG") == "0":  # A/B only: the separate level-0 conv1 weight-gradient launch
        net.ln_wg = False
    if os.environ.get("NBP_FFN_ROWS") == "0":  # A/B only: the deep-level FFN half as separate launches
        net.fuse_ffn_rows = False
    return NBPTrainer(net, psf_mode="rgb", psf_spec=spec, **wl["w"]), init_sd


def batch(dev, B, img, rank):
    g = torch.Generator(device=dev).manual_seed(0 + rank)
    lq = torch.rand(B, 3, img, img, device=dev, generator=g)
    gt = torch.rand(B, 3, img, img, device=dev, generator=g)
    ratio = torch.ones(B, 1, 1, 1, device=dev)
    return lq, gt, (lq * ratio).clamp(0, 1), ratio


def raw_metric(tr, b, ratios):
    """cfg5's linear-domain metric on the trainer's last output: phys_cons_raw(pred, short, psf, expo_ratio)
    (metrics/phys_consistency.py:193-320: y_hat = psf * pred, times the ratio, against the observation, valid crop),
    fp16 inputs (the metric accumulates in fp32, phys_consistency.py:302-303).  The observation is built from the bench
    batch's ground truth with the SAME forward model and ratios (obs = ratio * psf(gt), reflect padding), so that
    phys_cons_raw(gt, obs) is ~0 (`gt_mean`, the fp16 rounding of the inputs) and the value for the output measures its
    distance from the physically consistent image; the training step itself runs on the bench's own synthetic pair."""
    import torch.nn.functional as Fn
    from lowlight_image_enhancement_amd.metrics.phys_consistency import phys_cons_raw
    out = tr._graph_out if getattr(tr, "_graph", None) is not None else None
    if out is None:
        out = tr.net(b[0])
    B = out.shape[0]
    r = torch.tensor([ratios[i % len(ratios)] for i in range(B)], device=out.device)
    k = tr.kernel  # [3, 1, 3, 3] depthwise crosstalk PSF -> the metric's [C_out, C_in, 3, 3] form (diagonal)
    psf = torch.zeros(k.shape[0], k.shape[0], k.shape[2], k.shape[3], device=k.device)
    for c in range(k.shape[0]):
        psf[c, c] = k[c, 0]
    gt = b[1].float()
    kn = k / k.sum(dim=(2, 3), keepdim=True)  # the metric's normalize_psf (the trainer's kernel is normalised already)
    obs = Fn.conv2d(Fn.pad(gt, (1, 1, 1, 1), mode="reflect"), kn, groups=k.shape[0]) * r.view(B, 1, 1, 1)
    obs = obs.half()
    per = phys_cons_raw(out.detach().clamp_min(0).half(), obs, psf, r, reduction="none")
    per_gt = phys_cons_raw(gt.half(), obs, psf, r, reduction="none")
    return {"mean": round(float(per.mean()), 6), "per_image": [round(float(v), 6) for v in per.flatten()],
            "gt_mean": round(float(per_gt.mean()), 6), "expo_ratio": [float(v) for v in r.tolist()],
            "obs": "ratio * psf(gt) (reflect pad), fp16", "inputs": "fp16 (output clamp_min 0)"}


def short_run(dev, workload, precision, steps=5, warmup=3):
    """img/s of a graph-replayed run (extra keys; the headline is the main run)."""
    wl = WORKLOADS[workload]
    tr, _ = make_trainer(dev, workload, precision)
    b = batch(dev, wl["batch"], wl["img"], 0)
    for _ in range(warmup):
        tr.graph_step(*b)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.graph_step(*b)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    out = {"value": round(wl["batch"] / dt, 2), "unit": "img/s", "ms_per_step": round(dt * 1e3, 3),
           "precision": precision, "steps": steps, "warmup": warmup, "losses": tr.logs()}
    if "raw_ratios" in wl:
        out["phys_cons_raw"] = raw_metric(tr, b, wl["raw_ratios"])
    del tr
    torch.cuda.empty_cache()
    return out


def plan_launch(gpus, env, device_count, rehearse):
    """How this invocation runs, from `--gpus` (None = not given) and the launcher environment:
    ("run", world) = this process is one rank of `world` (a launcher set WORLD_SIZE, or N = 1);
    ("spawn", N)   = start N local ranks (WORLD_SIZE unset, N > 1).
    Raises SystemExit with a message when the request cannot be honoured: WORLD_SIZE != --gpus, N < 1, or fewer
    visible GPUs than N (unless rehearsing on one GPU)."""
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        world = int(ws)
        if gpus is not None and gpus != world:
            raise SystemExit(f"bench.py: --gpus {gpus} but the launcher started WORLD_SIZE={world} ranks; they must match")
        return "run", world
    n = 1 if gpus is None else gpus
    if n < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1, got {n}")
    if not rehearse and device_count < n:
        raise SystemExit(f"bench.py: --gpus {n} requested but only {device_count} GPU(s) are visible")
    return ("spawn", n) if n > 1 else ("run", 1)


def rank_envs(n, base_env, port):
    """The environment of each of n local ranks (torchrun's variables; MASTER_ADDR 127.0.0.1)."""
    envs = []
    for r in range(n):
        e = dict(base_env)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        envs.append(e)
    return envs


def spawn_ranks(n, argv):
    """Start n copies of this script as local ranks (child processes: no exec, no GPU call in this parent), wait for
    all, and return the first non-zero exit status (the others are then terminated by PID)."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=e)
             for e in rank_envs(n, os.environ, port)]
    status = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and status == 0:
                status = rc
                print(f"[bench] rank {procs.index(p)} exited with status {rc}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                for q in live:
                    q.terminate()
        time.sleep(0.2)
    return status


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="GPUs = ranks (default: WORLD_SIZE under a launcher, else 1)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--quick", action="store_true", help="headline only: no extra modes / cfg3 / CPU baseline")
    ap.add_argument("--eager", action="store_true", help="time eager launches instead of HIP-graph replays")
    ap.add_argument("--precision", default="fp16", choices=["fp16", "bf16", "fp32"],
                    help="fp16 (default; the reference's AMP dtype) / bf16: 16-bit storage + MFMA operands, fp32 "
                         "accumulation; fp32: fp32 everywhere (parity mode)")
    ap.add_argument("--workload", default="cfg2", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=0, help="per-GPU batch override (diagnostics; 0 = the workload's)")
    args = ap.parse_args()
    wl = WORKLOADS[args.workload]
    BATCH, IMG = (args.batch or wl["batch"]), wl["img"]

    # NBP_BENCH_REHEARSE=1 (one-GPU box only, never the measurement): every rank on cuda:0 over gloo, to exercise the
    # N > 1 path (graph segments + bucket all-reduces, barriers, max-over-ranks timing) where RCCL needs one GPU per rank
    rehearse = os.environ.get("NBP_BENCH_REHEARSE") == "1"
    # counting devices does not initialise the GPU on this image (its documented behaviour; the parent of spawned ranks
    # makes no other GPU call and starts its ranks as child processes, no exec; success path recorded in
    # profiles/r05_rehearsal/)
    how, world = plan_launch(args.gpus, os.environ, torch.cuda.device_count(), rehearse)
    if how == "spawn":
        sys.exit(spawn_ranks(world, sys.argv[1:]))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if rehearse:
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from lowlight_image_enhancement_amd import _lib

    tr, init_sd = make_trainer(dev, args.workload, args.precision)
    net = tr.net
    lq, gt, short, ratio = batch(dev, BATCH, IMG, rank)

    for _ in range(args.warmup):
        tr.step(lq, gt, short, ratio)
    tr.logs()

    # live per-launch timing (HIP events on the launch stream) over K eager steps; each record carries the launch's
    # algorithmic FLOPs and HBM bytes (operands read once, outputs written once)
    prof = {}

    def mk(records):
        def cb(a, e0, e1):
            for cls, fl, by, nl, slab in records(a):
                prof.setdefault(cls, []).append((fl, by, nl, slab, e0, e1))
        return cb

    for name, records in ENTRIES.items():
        _lib.PROFILE[name] = mk(records)
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
    step_events = []
    _lib.launch_timing(True)  # the one-kernel classes: events around each of their launches inside the library
    tr.comm_probe = world > 1  # the eager steps' exposed all-reduce time (not NAFBlock time, not the rest either)
    for _ in range(args.steps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        tr.step(lq, gt, short, ratio)
        e1.record()
        step_events.append((e0, e1))
    torch.cuda.synchronize()
    _lib.PROFILE.clear()
    inst = {}
    for name, ms_, fl_, by_ in _lib.launch_timing_records():
        if name in INSTANCES:
            v = inst.setdefault(INSTANCES[name], [0.0, 0.0, 0.0, 0, 0, 0.0])
            v[0] += ms_; v[1] += fl_; v[2] += by_; v[3] += 1; v[4] += 1  # noqa: E702
    _lib.launch_timing(False)
    net._block_fwd, net._block_bwd = orig_fwd, orig_bwd
    eager_comm = tr.comm_stats() if world > 1 else None
    tr.comm_probe, tr.comm_events = False, []

    # graph replay at every world size (N > 1: segments cut at the gradient buckets, all-reduces between them); a
    # rank whose capture fails falls back to eager steps, which issue the same collective sequence
    use_graph = not args.eager
    run = tr.graph_step if use_graph else tr.step
    if use_graph:
        try:
            run(lq, gt, short, ratio)  # capture + one replay, untimed
        except Exception as e:  # noqa: BLE001
            print(f"[bench] rank {rank}: graph capture failed ({type(e).__name__}: {e}); eager steps", file=sys.stderr)
            tr._graph = None
            use_graph, run = False, tr.step
            torch.cuda.synchronize()
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
    comm = None
    if world > 1:
        # after the timed region: a few probed steps of the same kind (events on the compute stream around the bucket
        # waits, after the last backward segment) -> the all-reduce time the backward left exposed
        tr.comm_probe = True
        for _ in range(min(args.steps, 5)):
            run(lq, gt, short, ratio)
        comm = tr.comm_stats()
        tr.comm_probe, tr.comm_events = False, []
        comm["allreduce_exposed_ms_eager"] = eager_comm["allreduce_exposed_ms"]
        comm["note"] = ("exposed = compute-stream time from the end of the last backward kernel to the completion of "
                        "every bucket all-reduce (graph replays; _eager: the profiled eager steps); rank 0's view")
    logs = tr.logs()

    classes = {}
    for cls, recs in prof.items():
        ms = sum(e0.elapsed_time(e1) for *_, e0, e1 in recs)
        classes[cls] = (ms, sum(r[0] for r in recs), sum(r[1] for r in recs), sum(r[2] for r in recs), len(recs),
                        sum(r[3] for r in recs))
    classes.update({k: tuple(v) for k, v in inst.items()})
    # the dominant KERNEL: the one-instance line with the most time per step
    dom = max((k for k in classes if k in SINGLE_KERNEL), key=lambda k: classes[k][0])
    ms, fl, by, nl, _, _ = classes[dom]
    peak_tf = FP32_PEAK_TFLOPS if args.precision == "fp32" else MFMA16_PEAK_TFLOPS
    tflops = fl / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
    gbps = by / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    # the binding roof is the one the class is closer to (arithmetic intensity vs the ridge point)
    if fl / max(by, 1) < peak_tf * 1e12 / (HBM_PEAK_GBPS * 1e9):
        roof = {"bound": "hbm", "achieved": round(gbps, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(gbps / HBM_PEAK_GBPS, 4)}
    else:
        roof = {"bound": "mfma", "achieved": round(tflops, 3), "peak": peak_tf, "unit": "TFLOP/s",
                "frac": round(tflops / peak_tf, 4)}
    traffic, tsrc = _pmc_traffic(dom)
    roof.update({"traffic": traffic, "traffic_source": tsrc, "kernel": dom,
                 "rocprof_kernels": [r.format(T=MANGLED_T[args.precision]) for r in ROCPROF_KERNELS[dom]],
                 "timing": "HIP events around each launch of this instance inside the library (nbp_launch_timing), "
                           "eager profiled steps",
                 "launches_per_step": round(nl / args.steps, 2), "ms_per_step": round(ms / args.steps, 3),
                 "avg_launch_us": round(ms * 1e3 / nl, 2), "algorithmic_bytes_per_launch": round(by / max(nl, 1)),
                 "algorithmic_bytes_per_step": round(by / args.steps),
                 "traffic_over_algorithmic": None if traffic is None else round(traffic / max(by / max(nl, 1), 1), 3),
                 "algorithmic_bytes_definition": UNIT_DEF[dom],
                 "algorithmic_flops_per_launch": round(fl / max(nl, 1)), "flop_intensity": round(fl / max(by, 1), 2),
                 "tflops": round(tflops, 2), "mfma_frac": round(tflops / peak_tf, 4),
                 "classes": {k: _class_line(k, v, args.steps, peak_tf, MANGLED_T[args.precision])
                             for k, v in classes.items()}})
    # the next instance by time per step: within a few % of the dominant one, the two can swap places between runs and
    # between this live timing and a rocprof summary (per-dispatch serialisation), so the line names both
    ranked = sorted((k for k in classes if k in SINGLE_KERNEL), key=lambda k: -classes[k][0])
    if len(ranked) > 1:
        ru, rl = ranked[1], roof["classes"][ranked[1]]
        roof["runner_up"] = {"kernel": ru, "ms_per_step": rl.get("ms_per_step"), "hbm_frac": rl.get("hbm_frac"),
                             "mfma_frac": rl.get("mfma_frac"),
                             "ms_ratio_to_dominant": round(classes[ru][0] / max(classes[dom][0], 1e-9), 3)}
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
    esize = ESIZE[args.precision]
    blk_bytes = nafblock_bytes(net, BATCH, IMG, IMG, esize)
    # The eager per-block events include host-dispatch stalls at the small levels (the GPU outruns the launches
    # there); the NAFBlock GPU time is the timed step minus the non-NAFBlock part of the eager step (boundary convs,
    # down/up, loss head, optimizer: few large kernels, not dispatch-bound).
    step_ms = elapsed / args.steps * 1e3
    # N > 1: the exposed all-reduce time is neither NAFBlock nor the rest of the step: it leaves the eager
    # non-block part and the timed step alike
    exp_eager = (eager_comm or {}).get("allreduce_exposed_ms") or 0.0
    exp_graph = (comm or {}).get("allreduce_exposed_ms") or 0.0
    nonblock_ms = max(eager_step_ms - blk_ms - exp_eager, 0.0)
    blk_ms_gpu = max(step_ms - exp_graph - nonblock_ms, 1e-6)
    blk_gbps = blk_bytes / (blk_ms_gpu * 1e-3) / 1e9

    if rank == 0:
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
            "config": {"workload": wl["desc"], "global_batch": BATCH * world, "image": IMG,
                       "parallelism": f"dp{world}", "precision": args.precision,
                       "launch": "hip-graph replay" if use_graph else "eager",
                       **({"rehearsal": "gloo, every rank on cuda:0 (not a measurement)"} if rehearse else {})},
            "roofline": roof,
            "nafblock_roofline": {"bytes_per_step": blk_bytes, "bytes_per_element": esize,
                                  "ms_per_step": round(blk_ms_gpu, 3),
                                  "ms_method": "timed step - non-NAFBlock part of the eager step" + (
                                      " (both net of their exposed all-reduce time)" if world > 1 else ""),
                                  "eager_blocks_ms_per_step": round(blk_ms, 3),
                                  "per_level_eager": per_level,
                                  "achieved_GBps": round(blk_gbps, 1), "peak_GBps": HBM_PEAK_GBPS,
                                  "frac": round(blk_gbps / HBM_PEAK_GBPS, 4)},
            "losses": logs,
        }
        if comm is not None:
            res["comm"] = comm
        if "raw_ratios" in wl:
            res["phys_cons_raw"] = raw_metric(tr, (lq, gt, short, ratio), wl["raw_ratios"])
        if world == 1:
            res["psnr_vs_cpu_ref_db"], res["max_abs_vs_cpu_ref"] = psnr_vs_cpu(net, dev, IMG)
            res["psnr_active_blocks_db"], res["max_abs_active_blocks"] = psnr_vs_cpu(net, dev, IMG, active=True)
            if not args.quick and args.workload == "cfg2":
                del tr, net
                torch.cuda.empty_cache()
                print("[bench] extra modes", file=sys.stderr, flush=True)
                res["modes"] = {p: short_run(dev, "cfg2", p) for p in ("fp32", "bf16", "fp16") if p != args.precision}
                print("[bench] cfg3 sample", file=sys.stderr, flush=True)
                res["cfg3"] = dict(short_run(dev, "cfg3", args.precision, steps=3, warmup=2),
                                   workload=WORKLOADS["cfg3"]["desc"], global_batch=WORKLOADS["cfg3"]["batch"])
                print("[bench] cfg4 N=1 line", file=sys.stderr, flush=True)
                res["cfg4"] = dict(short_run(dev, "cfg4", args.precision, steps=5, warmup=3),
                                   workload=WORKLOADS["cfg4"]["desc"], global_batch=WORKLOADS["cfg4"]["batch"],
                                   note="the >= 6.5x scaling config at N = 1 (python bench.py --workload cfg4 "
                                        "--gpus N starts N local ranks and times it at N GPUs)")
                print("[bench] cfg5 N=1 line", file=sys.stderr, flush=True)
                res["cfg5"] = dict(short_run(dev, "cfg5", args.precision, steps=3, warmup=2),
                                   workload=WORKLOADS["cfg5"]["desc"], global_batch=WORKLOADS["cfg5"]["batch"],
                                   note="BASELINE configs[4] per GPU (4 x 8 = bs 32 globally); python bench.py "
                                        "--workload cfg5 --gpus 4 times it at 4 GPUs")
                if not args.no_cpu_baseline:
                    print("[bench] cpu baseline", file=sys.stderr, flush=True)
                    res["cpu_baseline"] = cpu_baseline(init_sd)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
