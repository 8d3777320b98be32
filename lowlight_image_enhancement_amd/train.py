"""Fused training step on MI355X — the hot path of ImageRestorationModel.optimize_parameters
(NAFNet_base/basicsr/models/image_restoration_model.py:247-322, fp32 branch :316-320) with the HybridLossPlus term
wiring of the configs (NewBP_model/losses.py:318-372, configs/colab/sid_newbp_rgb.yml:78-96):

    out = net(lq) ; L = w_l1*L1(out, gt) + w_ssim*SSIM(out01, gt01) + w_phys*Phys_srgb(out01, short01, ratio)
    backward ; [all-reduce grads / world] ; clip_grad_norm_(0.01) ; AdamW(lr, (0.9, 0.999), wd 0.01)

Everything runs as HIP kernels on the current stream: the executor of nafnet.py, the loss kernels (clamp(0,1) of
the caller, :298-300, is fused into them), the global-norm clip and AdamW over the flat parameter buffer.  No host
synchronisation inside a step: loss values stay on the device until `logs()` is read.

Data parallel (one process per GPU, torch.distributed 'nccl' = RCCL): the backward executor reports each stage
whose gradient slice is complete; stages are packed into ~bucket_mb buckets that are all-reduced asynchronously
(SUM) while the backward continues, the 1/world average is folded into the clip kernel.  The initial parameters are
broadcast from rank 0 (the DDP construction broadcast, base_model.py:72-78).

Deliberate differences, all numerically neutral: the `0.0 * sum(p.sum())` term (:306) is omitted (its value and
gradient are exactly zero for finite parameters); the per-term `_ensure_finite` host syncs (losses.py:298-306)
become one device-side finiteness flag checked when logs are read; the loss dict is reduced with an all-reduce
instead of reduce-to-rank-0 (:351).
"""
from __future__ import annotations

import math
import struct
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from . import _lib
from ._lib import call, query
from .NewBP_model.losses import _ratio_array
from .NewBP_model.newbp_layer import build_psf_kernels, normalize_kernels
from .nafnet import NAFNet, Stage


class TrueCosineAnnealingLR:
    """lr(t) = eta_min + (base - eta_min) * (1 + cos(pi * t / T_max)) / 2 (configs .../sid_newbp_rgb.yml:74-77)."""

    def __init__(self, base_lr: float, T_max: int, eta_min: float = 0.0):
        self.base, self.T, self.eta_min = base_lr, T_max, eta_min

    def __call__(self, t: int) -> float:
        return self.eta_min + (self.base - self.eta_min) * (1 + math.cos(math.pi * t / self.T)) / 2


class NBPTrainer:
    def __init__(self, net: NAFNet, psf_mode: str = "rgb", psf_spec: str = "B2", w_l1: float = 1.0,
                 w_ssim: float = 0.0, w_phys: float = 0.1, lr: float = 5e-4, betas=(0.9, 0.999),
                 weight_decay: float = 0.01, eps: float = 1e-8, max_norm: Optional[float] = 0.01,
                 scheduler: Optional[TrueCosineAnnealingLR] = None, process_group=None, bucket_mb: float = 25.0,
                 w_deltaE: float = 0.0, w_perc: float = 0.0, w_lpips: float = 0.0, perceptual=None, lpips=None,
                 loss_scale: Optional[str] = "auto", init_scale: float = 2.0 ** 16, growth_factor: float = 2.0,
                 backoff_factor: float = 0.5, growth_interval: int = 2000, lpips_net: str = "vgg",
                 data_parallel: Optional[bool] = None):
        """Loss terms and weights as HybridLossPlus (losses.py:223-372): L1 (raw), Perc (VGG19), LPIPS (vgg), ΔE00,
        SSIM, Phys_srgb; a zero weight skips the term.  `perceptual` / `lpips`: PerceptualLoss / LPIPS modules
        (constructed with the synthetic offline weights when needed and not given; `lpips_net` picks the backbone of
        a constructed LPIPS: 'vgg' as HybridLossPlus, or 'alex' as BASELINE.json cfg3 names it).  `loss_scale`: "auto" (dynamic
        GradScaler scaling when net.precision == "fp16"), "dynamic" or None; the GradScaler arguments are torch's
        defaults.  A step whose gradient is non-finite leaves parameters and moments untouched in every mode."""
        self.net = net
        dev = net.flat.device
        self.dev = dev
        self.kernel = normalize_kernels(build_psf_kernels(psf_mode, psf_spec)).to(dev)
        self.k_shared = int(psf_mode == "mono")
        self.w = (float(w_l1), float(w_ssim), float(w_phys))
        self.w_extra = dict(de=float(w_deltaE), perc=float(w_perc), lpips=float(w_lpips))
        # upstream gradients of the loss terms, read by the kernels from device memory: up = up_base * S (the loss
        # scale), {L1, SSIM, Phys, DeltaE, Perc} then one LPIPS entry per image (d(w * mean_n LPIPS_n) / d LPIPS_n)
        self.up_base: Optional[torch.Tensor] = None
        self.up: Optional[torch.Tensor] = None
        self._ups: Dict[int, tuple] = {}  # batch size -> (up_base, up), never freed (graphs hold their addresses)
        if w_perc and perceptual is None:
            from .NewBP_model.losses import PerceptualLoss
            perceptual = PerceptualLoss(device=dev)
        if w_lpips and lpips is None:
            from .lpips import LPIPS
            lpips = LPIPS(net=lpips_net)
        self.perceptual, self.lpips = perceptual, lpips
        self.lpips_buf: Optional[torch.Tensor] = None
        self._lpips_bufs: Dict[int, torch.Tensor] = {}  # batch size -> per-image LPIPS values, never freed (as _ups)
        self._skipped_seen = 0  # ctl[2] (skipped steps) at the previous logs() call
        self.lr, self.betas, self.wd, self.eps = lr, betas, weight_decay, eps
        self.max_norm = max_norm if max_norm is not None else 0.0
        self.scheduler = scheduler
        n = net.numel
        self.grad = torch.zeros(n, device=dev)
        self.exp_avg = torch.zeros(n, device=dev)
        self.exp_avg_sq = torch.zeros(n, device=dev)
        self.clip_ws = torch.empty(query("clip_workspace_doubles", n), dtype=torch.float64, device=dev)
        # device-side step state (nbp_optim_prepare): state = {norm, grad multiplier, skip, lr/bc1, sqrt(bc2), lr, S},
        # ctl = {AdamW steps taken, GradScaler growth tracker, skipped steps}
        self.opt_state = torch.zeros(8, device=dev)
        self.ctl = torch.zeros(4, dtype=torch.int32, device=dev)
        self._lr_dev = torch.zeros(1, device=dev)
        # GradScaler (image_restoration_model.py:104-106, torch.cuda.amp defaults): dynamic loss scaling whenever the
        # activations are stored in fp16 (the reference's autocast dtype); fp32 / bf16 need none (8-bit exponent)
        if loss_scale == "auto":
            loss_scale = "dynamic" if net.precision == "fp16" else None
        self.scaler = (torch.tensor([init_scale, growth_factor, backoff_factor, float(growth_interval)],
                                    dtype=torch.float32, device=dev) if loss_scale == "dynamic" else None)
        # VGG / LPIPS trunk type for modules left at precision "auto" (the trainer's default ones): fp32 in the fp32
        # parity mode (the reference's fp32 trunk); in the 16-bit modes the autocast counterpart -- fp16 only under a
        # loss scale (its ~1/n feature gradients underflow fp16 otherwise), else bf16.  A module given an explicit
        # precision keeps it; the trainer never changes a module's attributes.
        self.vgg_dt = 0 if net.precision == "fp32" else (2 if net.precision == "fp16" and self.scaler is not None else 1)
        self.loss_buf = torch.zeros(6, device=dev)  # L1, SSIM, Phys, DeltaE, Perc, Total
        self.iter = 0  # iterations run (the scheduler's position; AdamW's own step count self.t excludes skips)
        self.pg = process_group
        have_pg = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(process_group) if have_pg else 1
        # the bucketed all-reduce path (per-stage hooks, asynchronous bucket all-reduces, graph segments cut at the
        # buckets): on whenever world > 1; data_parallel=True forces it on a one-rank process group too (the RCCL
        # rehearsal of the path on one GPU: a one-rank SUM all-reduce is the identity, so the step is bitwise the
        # non-data-parallel one)
        if data_parallel and not have_pg:
            raise ValueError("data_parallel=True needs an initialised torch.distributed process group")
        self.dp = self.world > 1 if data_parallel is None else bool(data_parallel)
        self.bucket_elems = int(bucket_mb * 1024 * 1024 / 4)
        self._handles: List = []
        self._cap: Optional[dict] = None  # segment capture state of the data-parallel graph step
        self._pending_lo: Optional[int] = None
        self._pending_hi = 0
        # communication accounting (the N > 1 bench line): buckets and bytes all-reduced by the last step, and, while
        # comm_probe is set, a pair of events per step on the compute stream -- after the last backward kernel (the
        # last graph segment) and after the waits for every bucket's all-reduce: the all-reduce time left exposed
        self.comm_buckets: List[tuple] = []
        self.comm_probe = False
        self.comm_events: List[tuple] = []
        if self.dp:
            dist.broadcast(net.flat.data, src=0, group=process_group)

    # ------------------------------------------------------------------ bucketed all-reduce during backward
    def _on_stage(self, st: Stage):
        if self._pending_lo is None:
            self._pending_lo = st.lo
        self._pending_hi = st.hi
        if self._pending_hi - self._pending_lo >= self.bucket_elems:
            self._flush()

    def _flush(self):
        if self._pending_lo is None or self._pending_hi <= self._pending_lo:
            return
        lo, hi = self._pending_lo, self._pending_hi
        self._pending_lo = None
        if self._cap is not None:  # capturing graph segments: cut here; the replay all-reduces between segments
            self._cut_segment((lo, hi))
            return
        self.comm_buckets.append((lo, hi))
        h = dist.all_reduce(self.grad[lo:hi], op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
        self._handles.append(h)

    def _wait_buckets(self):
        """Wait (on the current stream) for every bucket all-reduce issued this step; with comm_probe set, events
        bracket the wait: their distance is the all-reduce time the backward did not hide."""
        e0 = None
        if self.comm_probe:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        for h in self._handles:
            h.wait()
        self._handles.clear()
        if e0 is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            self.comm_events.append((e0, e1))

    def comm_stats(self) -> Dict[str, float]:
        """Buckets and gradient bytes all-reduced per step (the last step's), and the mean exposed all-reduce time of
        the probed steps (ms; None when none was probed).  Reference contract: the DDP gradient all-reduce
        (base_model.py:72-78, basicsr/train.py:54-63)."""
        if self.comm_events:
            torch.cuda.synchronize()
        exp =[a.elapsed_time(b) for a, b in self.comm_events]
        return {"buckets_per_step": len(self.comm_buckets),
                "bytes_allreduced_per_step": int(sum(hi - lo for lo, hi in self.comm_buckets) * 4),
                "bucket_mb": round(self.bucket_elems * 4 / 2 ** 20, 3),
                "allreduce_exposed_ms": round(sum(exp) / len(exp), 4) if exp else None,
                "probed_steps": len(exp)}

    def _cut_segment(self, bucket):
        """End the graph segment being captured (its last kernels complete `bucket`'s gradient slice) and begin the
        next one in the same memory pool."""
        cap = self._cap
        cap["g"].capture_end()
        cap["segs"].append((cap["g"], bucket))
        cap["g"] = torch.cuda.CUDAGraph()
        cap["g"].capture_begin(pool=cap["pool"], capture_error_mode=cap["mode"])

    # ------------------------------------------------------------------ the step
    def loss_and_grad(self, lq, gt, short=None, expo_ratio=None):
        """Forward + loss head + backward into self.grad (no optimizer update)."""
        net = self.net
        _lib.require_cuda(lq, gt)
        lq, gt = lq.contiguous(), gt.contiguous()
        B, C, H, W = lq.shape
        self._ensure_up(B)
        out, tape = net.exec_forward(lq, save=True)
        n = out.numel()
        wl1, wss, wph = self.w
        d_out = torch.empty_like(out)
        tmp = torch.empty_like(out)
        pix_ws = torch.empty(query("pix_workspace_doubles", n), dtype=torch.float64, device=lq.device)
        call("pix_loss_fwd", out, gt, n, 0, 0.0, 0, 0, pix_ws, self.loss_buf[0:1])
        call("pix_loss_bwd", out, gt, n, 0, 0.0, 0, 0, self.up[0:1], d_out)
        if wss != 0.0:
            ss_ws = torch.empty(query("ssim_workspace_floats", n), device=lq.device)
            call("ssim_loss_fwd", out, gt, B, C, H, W, 11, 1.0, 1, 1, 0, ss_ws, self.loss_buf[1:2], None)
            call("ssim_loss_bwd", out, gt, B, C, H, W, 1, self.up[1:2], None, ss_ws, tmp)
            call("add", d_out, tmp, d_out, n, 0)
        if wph != 0.0 and short is not None:
            if expo_ratio is None:  # ones [B,1,1,1] when the batch has no ratio (image_restoration_model.py:281-287)
                expo_ratio = torch.ones(B, 1, 1, 1, device=lq.device)
            r, full = _ratio_array(expo_ratio, short)
            ph_ws = torch.empty(query("phys_l1_workspace_doubles", B, C, H, W), dtype=torch.float64, device=lq.device)
            sign = torch.empty_like(out)
            call("phys_l1_fwd", out, short.contiguous(), r, full, self.kernel, self.k_shared, B, C, H, W, 3, 3, 0, 1, 1,
                 1, ph_ws, self.loss_buf[2:3], sign)
            call("phys_l1_bwd", sign, out, self.kernel, self.k_shared, self.up[2:3], B, C, H, W, 3, 3, 0, 1, tmp)
            call("add", d_out, tmp, d_out, n, 0)
        wde, wpe, wlp = self.w_extra["de"], self.w_extra["perc"], self.w_extra["lpips"]
        if wde != 0.0:
            de_ws = torch.empty(query("de00_workspace_doubles", B * H * W), dtype=torch.float64, device=lq.device)
            call("de00_loss_fwd", out, gt, B, H, W, 1, 1e-6, de_ws, self.loss_buf[3:4])
            call("de00_loss_bwd", out, gt, B, H, W, 1, 1e-6, self.up[3:4], tmp)
            call("add", d_out, tmp, d_out, n, 0)
        if wpe != 0.0:
            g = self.perceptual.value_and_grad(out, gt, self.up[4:5], self.loss_buf[4:5], dt=self._trunk_dt(self.perceptual))
            call("add", d_out, g, d_out, n, 0)
        if wlp != 0.0:
            g = self.lpips.value_and_grad(out, gt, self.up[5:5 + B], self.lpips_buf, clamp=True,
                                          dt=self._trunk_dt(self.lpips))
            call("add", d_out, g, d_out, n, 0)
        hook = self._on_stage if self.dp else None
        if self.dp and self._cap is None:
            self.comm_buckets = []
        net.exec_backward(tape, d_out, self.grad, need_dx=False, hook=hook)
        if self.dp:
            self._flush()
            if self._cap is None:
                self._wait_buckets()
        return out

    def _trunk_dt(self, module) -> Optional[int]:
        return self.vgg_dt if getattr(module, "precision", "auto") == "auto" else None

    def _ensure_up(self, B: int):
        """Select the upstream-gradient buffers of a batch of B images.  One pair (up_base, up) per batch size is kept
        for the trainer's lifetime: a captured graph addresses its pair by device pointer, so a pair is never freed or
        rebound.  Switching to another batch size refreshes that pair's up = up_base * S from the current loss scale
        (a device op: the optimizer of the steps run at other sizes moved S).  The per-image LPIPS value buffer is
        kept per batch size the same way (a captured graph's LPIPS tap kernels write into it)."""
        if self.up_base is not None and self.up_base.numel() == 5 + B:
            return
        if self.w_extra["lpips"]:
            buf = self._lpips_bufs.get(B)
            if buf is None:
                buf = self._lpips_bufs[B] = torch.zeros(B, device=self.dev)
            self.lpips_buf = buf
        pair = self._ups.get(B)
        if pair is None:
            wl1, wss, wph = self.w
            base = [wl1, wss, wph, self.w_extra["de"], self.w_extra["perc"]] + [self.w_extra["lpips"] / B] * B
            up_base = torch.tensor(base, dtype=torch.float32, device=self.dev)
            pair = self._ups[B] = (up_base, up_base.clone())
        self.up_base, self.up = pair
        self._refresh_up()

    def _refresh_up(self):
        """up = up_base * S (the loss scale on the device), or up_base without a scaler."""
        if self.up is None:
            return
        if self.scaler is not None:
            torch.mul(self.up_base, self.scaler[0], out=self.up)
        else:
            self.up.copy_(self.up_base)

    def _optimizer(self, grad_scale: float):
        """clip + finiteness verdict + GradScaler update (nbp_optim_prepare), then AdamW (nbp_adamw_apply)."""
        call("optim_prepare", self.grad, self.grad.numel(), float(grad_scale), float(self.max_norm), self.clip_ws,
             self._lr_dev, float(self.betas[0]), float(self.betas[1]), self.opt_state, self.ctl, self.scaler,
             self.up, self.up_base, self.up.numel())
        call("adamw_apply", self.net.flat.data, self.grad, self.exp_avg, self.exp_avg_sq, self.grad.numel(),
             self.opt_state, float(self.betas[0]), float(self.betas[1]), float(self.eps), float(self.wd))

    def _lr_now(self) -> float:
        """base_model.update_learning_rate (:164-174): iteration i (1-based) runs with the schedule at i - 1."""
        lr = self.scheduler(self.iter - 1) if self.scheduler is not None else self.lr
        return struct.unpack("f", struct.pack("f", lr))[0]

    @property
    def t(self) -> int:
        """AdamW steps taken (skipped non-finite steps excluded; a host sync)."""
        return int(self.ctl[0].item())

    @t.setter
    def t(self, v: int):
        self.ctl[0] = int(v)

    @property
    def skipped_steps(self) -> int:
        return int(self.ctl[2].item())

    def step(self, lq, gt, short=None, expo_ratio=None):
        out = self.loss_and_grad(lq, gt, short, expo_ratio)
        self.iter += 1
        self._lr_dev.fill_(self._lr_now())
        self._optimizer(1.0 / self.world)
        return out

    # ------------------------------------------------------------------ HIP-graph step
    def graph_step(self, lq, gt, short=None, expo_ratio=None):
        """One training step replayed from captured HIP graphs: every kernel of step() (forward, loss head,
        backward with its deferred reductions, clip, AdamW) recorded once and relaunched with no host work but the
        input copies and the lr upload.  Numerically identical to step().  The first call captures with these
        tensors' shapes; later calls copy their inputs into the captured buffers.

        Data parallel (world > 1): the step is captured as a chain of graph segments cut where the backward completes
        a gradient bucket; the replay launches each segment and then that bucket's asynchronous all-reduce (eager
        RCCL, outside any graph, so the collective overlaps the next segment exactly as in step()), waits for the
        buckets, and replays the clip + AdamW graph."""
        ins = (lq, gt, short, expo_ratio)
        if getattr(self, "_graph", None) is None:
            self._capture(ins)
        else:
            for dst, src in zip(self._static, ins):
                if (dst is None) != (src is None):
                    raise ValueError("graph_step: inputs must keep the structure of the captured step")
                if dst is not None and tuple(src.shape) != tuple(dst.shape):
                    raise ValueError(f"graph_step: input shape {tuple(src.shape)} differs from the captured "
                                     f"{tuple(dst.shape)}; use step() for other batch shapes")
            for dst, src in zip(self._static, ins):
                if dst is not None and src is not dst:
                    dst.copy_(src, non_blocking=True)
            self._ensure_up(self._static[0].shape[0])  # eager steps at another batch size may have switched pairs
        self.iter += 1
        slot = self.iter % len(self._lr_host)
        ev = self._lr_ev[slot]
        if ev is not None:
            ev.synchronize()  # the upload that last used this pinned slot has been consumed
        h = self._lr_host[slot]
        h[0] = self._lr_now()
        self._lr_dev.copy_(h, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._lr_ev[slot] = ev
        if not self.dp:
            self._graph.replay()
            return self._graph_out
        self.comm_buckets = []
        for g, bucket in self._segs:
            g.replay()
            if bucket is not None:
                lo, hi = bucket
                self.comm_buckets.append(bucket)
                self._handles.append(dist.all_reduce(self.grad[lo:hi], op=dist.ReduceOp.SUM, group=self.pg,
                                                     async_op=True))
        self._wait_buckets()
        self._graph.replay()  # clip (with the 1/world average) + AdamW
        return self._graph_out

    def _graph_body(self):
        lq, gt, short, ratio = self._static
        out = self.loss_and_grad(lq, gt, short, ratio)
        self._optimizer(1.0 / self.world)
        return out

    def _capture(self, ins):
        self._static = tuple(None if x is None else x.detach().clone() for x in ins)
        self._lr_host = [torch.zeros(1, pin_memory=True) for _ in range(8)]
        self._lr_ev = [None] * 8
        self._ensure_up(ins[0].shape[0])
        # the capture itself must not move any state: snapshot what the side-stream warm-up touches
        state = [self.net.flat.data, self.exp_avg, self.exp_avg_sq, self.ctl, self.opt_state, self.up] + (
            [self.scaler] if self.scaler is not None else [])
        saved = [x.clone() for x in state]
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            self._lr_dev.zero_()  # lazy initialisation happens outside the capture
            self._graph_body()
        torch.cuda.current_stream().wait_stream(side)
        for dst, src in zip(state, saved):
            dst.copy_(src)
        if not self.dp:
            self._graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._graph):
                self._graph_out = self._graph_body()
            return
        # data parallel: segments of fwd + bwd cut at every bucket flush (no collective inside any graph), then the
        # optimizer graph, all in one private memory pool and captured on one side stream
        torch.cuda.synchronize()
        pool = torch.cuda.graph_pool_handle()
        cs = torch.cuda.Stream()
        cs.wait_stream(torch.cuda.current_stream())
        # thread-local capture mode: the process group's watchdog thread may query events meanwhile
        mode = "thread_local"
        with torch.cuda.stream(cs):
            self._cap = {"pool": pool, "segs": [], "g": torch.cuda.CUDAGraph(), "mode": mode}
            live = False
            try:
                self._cap["g"].capture_begin(pool=pool, capture_error_mode=mode)
                live = True
                lq, gt, short, ratio = self._static
                out = self.loss_and_grad(lq, gt, short, ratio)
                live = False
                self._cap["g"].capture_end()
                self._cap["segs"].append((self._cap["g"], None))
                segs = self._cap["segs"]
                opt = torch.cuda.CUDAGraph()
                opt.capture_begin(pool=pool, capture_error_mode=mode)
                live = True
                self._optimizer(1.0 / self.world)
                live = False
                opt.capture_end()
            except BaseException:
                if live:  # leave the stream out of capture mode before re-raising
                    try:
                        (opt if "opt" in locals() else self._cap["g"]).capture_end()
                    except Exception:  # noqa: BLE001
                        pass
                raise
            finally:
                self._cap = None
        torch.cuda.current_stream().wait_stream(cs)
        torch.cuda.synchronize()
        self._segs, self._graph, self._graph_out = segs, opt, out

    def logs(self, reduce: bool = True) -> Dict[str, float]:
        """Loss dict of the last step (host sync), averaged over ranks like reduce_loss_dict (base_model.py:335-360)."""
        wl1, wss, wph = self.w
        wde, wpe, wlp = self.w_extra["de"], self.w_extra["perc"], self.w_extra["lpips"]
        buf = self.loss_buf.clone()
        lp = self.lpips_buf.mean().view(1) if (wlp and self.lpips_buf is not None) else torch.zeros(1, device=buf.device)
        buf = torch.cat([buf, lp])  # L1, SSIM, Phys, DeltaE, Perc, Total, LPIPS
        buf[5] = wl1 * buf[0] + wss * buf[1] + wph * buf[2] + wde * buf[3] + wpe * buf[4] + wlp * buf[6]
        if reduce and self.world > 1:
            dist.all_reduce(buf, group=self.pg)
            buf /= self.world
        vals = buf.cpu()
        skipped = int(self.ctl[2].item())
        new_skips, self._skipped_seen = skipped - self._skipped_seen, skipped  # counted once, even when raising below
        if not torch.isfinite(vals).all():
            raise RuntimeError(f"HybridLossPlus detected non-finite values: {vals.tolist()}")
        out = {"L1_raw": float(vals[0])}
        if wpe:
            out["Perc"] = float(vals[4])
        if wlp:
            out["LPIPS"] = float(vals[6])
        if wde:
            out["DeltaE"] = float(vals[3])
        if wss:
            out["SSIM"] = float(vals[1])
        if wph:
            out["Phys"] = float(vals[2])
        out["Total"] = float(vals[5])
        st = self.opt_state.cpu()
        out["grad_norm"] = float(st[0])
        if self.scaler is not None:
            out["loss_scale"] = float(st[6])
        if st[2] != 0 or new_skips > 0:
            if self.scaler is None:
                # no GradScaler: the reference has no skip here (image_restoration_model.py:316-320); a non-finite
                # gradient on ANY step since the previous logs() left the parameters untouched, and the run must not
                # continue silently
                raise RuntimeError(f"NBPTrainer: {max(new_skips, 1)} step(s) since the previous logs() had a non-finite "
                                   f"gradient (skipped; no loss scaler is active); last grad_norm={float(st[0])}")
            out["skipped"] = float(max(new_skips, 1))
        return out
