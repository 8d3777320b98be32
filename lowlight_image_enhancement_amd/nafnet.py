"""NAFNet (Scenario B) on MI355X: one flat fp32 parameter buffer + an executor over the HIP C-ABI.

Reference: NAFNet_base/basicsr/models/archs/NAFNet_arch.py:22-162 (NAFNet, NAFBlock, SimpleGate) and
arch_util.py:264-300 (LayerNorm2d).  Same constructor signature, same state_dict keys and tensor shapes
(checkpoints interchange with the reference); different internals:

* activations are NHWC between the intro and ending convs (channels contiguous for the 1x1 GEMMs, the
  per-pixel LayerNorm and the depthwise conv);
* all parameters live in ONE flat fp32 buffer (`self.flat`, the module's only nn.Parameter), laid out in
  reverse backward order so that gradient buckets for the data-parallel all-reduce are contiguous slices that
  complete in order; the optimizer, the global-norm clip and the all-reduce all run over that buffer;
* two weights are stored in the layout their kernels read: downs.i.weight as [2C][kh][kw][C] (the GEMM's K
  order over a space-to-depth gather) and ups.i.0.weight with its output rows grouped by PixelShuffle
  sub-position (r1, r2, c').  state_dict()/load_state_dict() convert to and from the reference layout.

The forward/backward executor launches the kernels of include/nbp.h on the current stream and keeps the
tensors the backward needs in a tape.
"""
from __future__ import annotations

import math
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

from . import _lib
from ._lib import call, query

AM_PLAIN, AM_S2D, AM_SCALE = 0, 1, 2
CM_SG, CM_SGBWD = 4, 5  # SimpleGate forward / backward fused into the GEMM epilogue (bf16 mode)
CM_CHANDOT = 8  # dgrad with the SCA channel-dot partials in the epilogue (bf16 mode, C > 64)
CM_PLAIN, CM_D2S = 0, 1
LN_EPS = 1e-6
# without a gradient-ready hook (one process: no bucketed all-reduce reads a stage's slice early) every deferred
# gradient reduction of the backward runs in the backward's final flush instead of one flush launch per stage: 26
# latency-bound reduce launches per step become a few full ones (+1.0 % at cfg2, fp16, in the quick bench: 1356 / 1358
# vs 1342 / 1344 img/s, gpurun_out r6c; the round-1 measurement of the same change was neutral).  NBP_LATE_FLUSH=0:
# per-stage flushes (A/B)
_LATE_FLUSH = __import__("os").environ.get("NBP_LATE_FLUSH", "1") != "0"


@dataclass
class PEntry:
    key: str
    ref_shape: Tuple[int, ...]
    offset: int
    numel: int
    kind: str = "plain"  # plain | down | up | sg (conv4: SimpleGate pairs interleaved)


@dataclass
class Stage:
    name: str
    lo: int  # flat offsets [lo, hi) of the parameters whose gradients this stage completes
    hi: int


def _block_keys(pre: str, c: int):
    return [(pre + "beta", (1, c, 1, 1)), (pre + "gamma", (1, c, 1, 1)),
            (pre + "conv1.weight", (2 * c, c, 1, 1)), (pre + "conv1.bias", (2 * c,)),
            (pre + "conv2.weight", (2 * c, 1, 3, 3)), (pre + "conv2.bias", (2 * c,)),
            (pre + "conv3.weight", (c, c, 1, 1)), (pre + "conv3.bias", (c,)),
            (pre + "sca.1.weight", (c, c, 1, 1)), (pre + "sca.1.bias", (c,)),
            (pre + "conv4.weight", (2 * c, c, 1, 1)), (pre + "conv4.bias", (2 * c,)),
            (pre + "conv5.weight", (c, c, 1, 1)), (pre + "conv5.bias", (c,)),
            (pre + "norm1.weight", (c,)), (pre + "norm1.bias", (c,)),
            (pre + "norm2.weight", (c,)), (pre + "norm2.bias", (c,))]


def _ceil_to(v, m):
    return (v + 3) // 4 * 4 if m == 4 else v


class NAFNet(nn.Module):
    """NAFNet(img_channel=3, width=16, middle_blk_num=1, enc_blk_nums=[], dec_blk_nums=[]) (NAFNet_arch.py:85)."""

    def __init__(self, img_channel=3, width=16, middle_blk_num=1, enc_blk_nums=[], dec_blk_nums=[]):  # noqa: B006
        super().__init__()
        if width < 4 or width % 4:
            raise ValueError("the MI355X NAFNet needs a width that is a multiple of 4 (16-byte channel vectors; the "
                             "16-bit precision modes need a multiple of 8)")
        if len(dec_blk_nums) != len(enc_blk_nums):
            raise ValueError("enc_blk_nums and dec_blk_nums must have the same length (U-Net skips)")
        if img_channel > 4:
            raise ValueError("img_channel <= 4")
        self.img_channel = img_channel
        self.width = width
        self.enc_blk_nums = list(enc_blk_nums)
        self.middle_blk_num = int(middle_blk_num)
        self.dec_blk_nums = list(dec_blk_nums)
        self.padder_size = 2 ** len(self.enc_blk_nums)
        self._build_layout()
        self.flat = nn.Parameter(torch.zeros(self.numel, dtype=torch.float32))
        self._init_reference_like()
        self.grad_ready_hook: Optional[Callable[[Stage], None]] = None
        self._keep: Optional[List[torch.Tensor]] = None  # slabs awaiting a deferred gradient reduction
        # Fused / folded forms of the executor, all on (each measured faster; the environment knobs that
        # toggled them for A/B runs were removed in round 4).  The attributes stay so that the GPU tests can compare
        # a fused form bit for bit with its unfused one on the same network.
        # LayerNorm forward in the conv3 / conv5 epilogues at C in {32, 64, 128, 256}
        self.fuse_ln_fwd = True
        # the wide (C >= 128) weight gradients of a whole U-Net level (conv5's U, conv4, conv3's U, conv1 of every
        # NAFBlock of the level) queued during the level's backward and launched as ONE grouped launch at its end,
        # with M-splits chosen for the group (False: one launch per weight gradient)
        self.group_wgrad = True
        self._grouping = False
        # level 0 (C = 32): the conv4 output t4 is not stored; the conv5 dgrad rebuilds it per tile on MFMA
        # (nbp_dgrad_sg_rc, bitwise equal) ...
        self.sg_rc = True
        # ... and folds conv5's U / V and conv4's weight / bias gradients into the same pass over dout / n2 / dt
        # (nbp_dgrad_sg_rc_wg; False: separate nbp_wgrad_f32 launches)
        self.sg_rc_wg = True
        # level 0 with that rebuild: conv4 -> SimpleGate -> conv5 (+ residual + next LayerNorm) as one pass
        # (nbp_gemm_ffn, bitwise the two launches, +0.1 % step), g2 never stored
        self.fuse_ffn = True
        # levels with C in {128, 256, 512} (16-bit): conv3 -> norm2 -> conv4 -> SimpleGate -> conv5 (-> the next norm1)
        # in one row-stationary launch (nbp_ffn_rows_fwd; bitwise the launches it replaces)
        self.fuse_ffn_rows = True
        # backward at those levels: a block's conv1 input gradient + norm1 backward deferred into the preceding block's
        # row-stationary launch (nbp_ffn_rows_bwd with dt1: its dx made in LDS as that block's dout; NBP_FFN_PRE=0 off)
        self.ffn_rows_pre = __import__("os").environ.get("NBP_FFN_PRE", "1") != "0"
        # levels with the stored tape: the SCA backward (ds, the SCA weight gradients) inside the fused depthwise
        # backward (nbp_sca_dw_bwd) instead of its own launch before it (NBP_SCA_FOLD=0: two launches)
        self.sca_fold = __import__("os").environ.get("NBP_SCA_FOLD", "1") != "0"
        # level 0: conv1's weight / bias gradients folded into the conv1 dgrad + norm1 backward pass (nbp_dgrad_ln_bwd_wg:
        # n1 rebuilt from x and the LN statistics, dt1 already in registers; False: a separate nbp_wgrad_f32 launch)
        self.ln_wg = True
        # the middle level (16 x 16 at C 512): conv1 -> depthwise -> SimpleGate -> pool as one whole-image launch
        # (nbp_c1_dw_sg_pool; t1 / t2 / g bitwise, the pool up to fp32 summation order)
        self.fuse_c1dw = True
        # levels 0 / 1 (C 32 / 64, 16-bit): conv1 -> depthwise -> SimpleGate -> pool as one row-walking tile launch that
        # keeps t1 / t2 on chip (nbp_c1dw_fwd_tile), and the mirror backward that rebuilds them from n1
        # (nbp_c1dw_bwd_tile): the 2C-wide tape never reaches HBM
        self.fuse_c1dw_tile = True
        # the levels (by channel count) that take it: 0 and 1.  The rebuild costs the backward more VALU work than the
        # stored-tape kernel (t1 epilogue + t2 recomputed: 172 vs 150 us at level 0, 102 vs 73 at level 1), which the
        # forward's saved tape traffic repays (58 vs 109 us, 49 vs 57): graph step +1.1 % with both levels, +0.7 / +0.3 %
        # with level 0 / 1 alone
        self.c1dw_tile_channels = (32, 64)
        self._ln_carry = None
        # "fp32": fp32 operands everywhere (parity mode); "fp16" / "bf16": 16-bit activation storage and MFMA operands
        # with fp32 accumulation, statistics, parameters and gradients (fp16 = the reference's AMP autocast dtype,
        # image_restoration_model.py:255; the trainer adds GradScaler-style dynamic loss scaling for it).
        self.precision = "fp32"
        # 16-bit modes: the layer scales beta / gamma are folded into the transposed conv3 / conv5 weight copies (the
        # dgrad operands: dh = (beta (.) dy) W3 = dy (diag(beta) W3)), so those dgrads read A unscaled
        self.fold_ls = True

        def _scale_off(k):
            if not self.fold_ls:
                return -1
            for wk, sk in (("conv3.weight", "beta"), ("conv5.weight", "gamma")):
                if k.endswith(wk):
                    return self.entries[k[:-len(wk)] + sk].offset
            return -1
        self._tdesc_cpu = torch.tensor([[e.offset, e.ref_shape[0], e.numel // e.ref_shape[0], _scale_off(k)]
                                        for k, e in self.entries.items() if self._is_gemm_weight(k)],
                                       dtype=torch.int64).reshape(-1, 4)
        self._tdesc = None
        # the weights nbp_ffn_rows_fwd / _bwd read (conv3 / conv4 / conv5, and conv1 for the backward's deferred input
        # gradient, of the levels with C in {128, 256, 512}), {offset, rows, cols}
        self._fdesc_cpu = torch.tensor([[e.offset, e.ref_shape[0], e.numel // e.ref_shape[0]]
                                        for k, e in self.entries.items()
                                        if k.endswith(("conv1.weight", "conv3.weight", "conv4.weight", "conv5.weight"))
                                        and e.numel // e.ref_shape[0] in (128, 256, 512)],
                                       dtype=torch.int64).reshape(-1, 3)
        self._fdesc = None

    # ------------------------------------------------------------------ layout
    def _build_layout(self):
        w = self.width
        # reference registration order (for state_dict key order)
        ref: List[Tuple[str, Tuple[int, ...]]] = [("intro.weight", (w, self.img_channel, 3, 3)), ("intro.bias", (w,)),
                                                  ("ending.weight", (self.img_channel, w, 3, 3)),
                                                  ("ending.bias", (self.img_channel,))]
        chan = w
        enc_keys, downs = [], []
        self.enc_chans = []
        for i, n in enumerate(self.enc_blk_nums):
            self.enc_chans.append(chan)
            for j in range(n):
                enc_keys += _block_keys(f"encoders.{i}.{j}.", chan)
            downs += [(f"downs.{i}.weight", (2 * chan, chan, 2, 2)), (f"downs.{i}.bias", (2 * chan,))]
            chan *= 2
        self.mid_chan = chan
        mid_keys = []
        for j in range(self.middle_blk_num):
            mid_keys += _block_keys(f"middle_blks.{j}.", chan)
        dec_keys, ups = [], []
        self.dec_chans = []
        for i, n in enumerate(self.dec_blk_nums):
            ups += [(f"ups.{i}.0.weight", (2 * chan, chan, 1, 1))]
            chan //= 2
            self.dec_chans.append(chan)
            for j in range(n):
                dec_keys += _block_keys(f"decoders.{i}.{j}.", chan)
        self.ref_order = [k for k, _ in ref + enc_keys + dec_keys + mid_keys + ups + downs]
        shapes = dict(ref + enc_keys + dec_keys + mid_keys + ups + downs)

        # flat layout in reverse backward order: ending, decoders (last first), ups, middle, enc/downs, intro
        # ending.bias (img_channel floats, not a multiple of 4) goes last so no alignment padding is needed and
        # the flat buffer holds exactly the reference's parameter count
        groups: List[Tuple[str, List[str]]] = [("ending", ["ending.weight"])]
        for i in reversed(range(len(self.dec_blk_nums))):
            for j in reversed(range(self.dec_blk_nums[i])):
                groups.append((f"decoders.{i}.{j}", [k for k, _ in _block_keys(f"decoders.{i}.{j}.", 1)]))
            groups.append((f"ups.{i}", [f"ups.{i}.0.weight"]))
        for j in reversed(range(self.middle_blk_num)):
            groups.append((f"middle_blks.{j}", [k for k, _ in _block_keys(f"middle_blks.{j}.", 1)]))
        for i in reversed(range(len(self.enc_blk_nums))):
            groups.append((f"downs.{i}", [f"downs.{i}.weight", f"downs.{i}.bias"]))
            for j in reversed(range(self.enc_blk_nums[i])):
                groups.append((f"encoders.{i}.{j}", [k for k, _ in _block_keys(f"encoders.{i}.{j}.", 1)]))
        groups.append(("intro", ["intro.weight", "intro.bias", "ending.bias"]))
        self.entries: Dict[str, PEntry] = OrderedDict()
        self.stages: Dict[str, Stage] = OrderedDict()
        off = 0
        for gname, keys in groups:
            lo = off
            for k in keys:
                shp = shapes[k]
                n = 1
                for s in shp:
                    n *= s
                kind = "down" if k.startswith("downs.") and k.endswith("weight") else (
                    "up" if k.startswith("ups.") else ("sg" if ".conv4." in k else "plain"))
                self.entries[k] = PEntry(k, shp, off, n, kind)
                off += n if k == "ending.bias" else _ceil_to(n, 4)  # 16-byte aligned slices for float4 access
            self.stages[gname] = Stage(gname, lo, off)
        self.numel = off

    @staticmethod
    def _is_gemm_weight(k: str) -> bool:
        return k.endswith(("conv1.weight", "conv3.weight", "conv4.weight", "conv5.weight")) or (
            k.startswith(("downs.", "ups.")) and k.endswith("weight"))

    def _prep_weights(self, P: torch.Tensor):
        """16-bit copy of the flat parameters + transposed copies of the GEMM weights (for the dgrads) + fragment-ordered
        copies of the deep levels' conv3 / conv4 / conv5 weights (nbp_ffn_rows_fwd; None when no level takes it)."""
        if self._tdesc is None or self._tdesc.device != P.device:
            self._tdesc = self._tdesc_cpu.to(P.device)
            self._fdesc = self._fdesc_cpu.to(P.device) if self._fdesc_cpu.shape[0] else None
            self._fdesc_t = self._fdesc_cpu[:, [0, 2, 1]].contiguous().to(P.device)  # the transposed copies: [in][out]
        wb = torch.empty(self.numel, dtype=self.adt, device=P.device)
        wt = torch.empty(self.numel, dtype=self.adt, device=P.device)
        call("weights_bf16", P, self.numel, wb, self._tdesc, self._tdesc.shape[0], wt, self.dt)
        wf = wtf = None
        if self.fuse_ffn_rows and self._fdesc is not None:  # fragment-ordered copies (nbp_frag16): forward, transposed
            wf = torch.empty(self.numel, dtype=self.adt, device=P.device)
            call("frag16", wb, self._fdesc, self._fdesc.shape[0], wf)
            wtf = torch.empty(self.numel, dtype=self.adt, device=P.device)
            call("frag16", wt, self._fdesc_t, self._fdesc_t.shape[0], wtf)
        return wb, wt, wf, wtf

    @property
    def adt(self) -> torch.dtype:
        """storage dtype of NHWC activations and activation gradients"""
        return {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}[self.precision]

    @property
    def dt(self) -> int:
        """dtype code of the C-ABI: 0 fp32, 1 bf16, 2 fp16"""
        d = {"fp32": 0, "bf16": 1, "fp16": 2}[self.precision]
        if d and self.width % 8:
            raise ValueError(f"precision {self.precision!r} needs a width that is a multiple of 8 (16-byte vectors of "
                             f"16-bit channels); width {self.width} runs in the fp32 mode")
        return d

    def _mm(self, W, A, lda, amode, ascale, rows, wkey, C, ldc, cmode, M, N, K, gh=0, gw=0, cs=0, bias=None,
            R=None, rscale=None, pre=None, dgrad=False):
        """One GEMM launch.  W = (fp32 flat,) or (fp32 flat, bf16 copy, bf16 transposed copy).
        forward: C[M,N] = A[M,K] . W[N,K]^T ; dgrad: C[M,N] = A[M,K] . W[K,N] (W stored [out=K][in=N])."""
        if len(W) == 1:
            Wf = self._slice(W[0], wkey)
            call("gemm_f32", A, lda, amode, ascale, rows, Wf, N if dgrad else K, 0 if dgrad else 1, C, ldc, cmode,
                 M, N, K, gh, gw, cs, bias, R, rscale, pre)
        else:
            Wb = self._slice(W[2] if dgrad else W[1], wkey)
            call("gemm_bf16", A, lda, amode, ascale, rows, self.dt, Wb, K, C, ldc, cmode, self.dt, M, N, K, gh, gw, cs,
                 bias, R, rscale, pre)

    # reference layout <-> internal layout
    def _to_internal(self, e: PEntry, t: torch.Tensor) -> torch.Tensor:
        if e.kind == "down":  # [2C, C, 2, 2] -> [2C, 2, 2, C]
            return t.permute(0, 2, 3, 1).reshape(-1)
        if e.kind == "sg":  # conv4 output rows h*C + c -> 2c + h: SimpleGate pairs adjacent (fused epilogues)
            n2 = t.shape[0]
            return t.reshape(2, n2 // 2, -1).permute(1, 0, 2).reshape(-1)
        if e.kind == "up":  # row n_ref = c'*4 + r1*2 + r2 -> n_int = (r1*2 + r2)*(C/2) + c'
            n2, c = t.shape[0], t.shape[1]
            return t.reshape(n2 // 4, 4, c).permute(1, 0, 2).reshape(-1)
        return t.reshape(-1)

    def _to_reference(self, e: PEntry, flat_slice: torch.Tensor) -> torch.Tensor:
        if e.kind == "sg":
            n2 = e.ref_shape[0]
            return flat_slice.view(n2 // 2, 2, -1).permute(1, 0, 2).reshape(e.ref_shape).contiguous()
        if e.kind == "down":
            o, c = e.ref_shape[0], e.ref_shape[1]
            return flat_slice.view(o, 2, 2, c).permute(0, 3, 1, 2).contiguous()
        if e.kind == "up":
            n2, c = e.ref_shape[0], e.ref_shape[1]
            return flat_slice.view(4, n2 // 4, c).permute(1, 0, 2).reshape(n2, c, 1, 1).contiguous()
        return flat_slice.view(e.ref_shape)

    def _slice(self, buf: torch.Tensor, key: str) -> torch.Tensor:
        e = self.entries[key]
        return buf[e.offset:e.offset + e.numel]

    def p(self, key: str) -> torch.Tensor:
        return self._slice(self.flat.data, key)

    @torch.no_grad()
    def _init_reference_like(self):
        """torch default init of the reference modules (Conv2d kaiming-uniform(a=sqrt(5)) weights and bias
        U(+-1/sqrt(fan_in)); LayerNorm2d ones/zeros; beta = gamma = 0, NAFNet_arch.py:56-57)."""
        for k, e in self.entries.items():
            leaf = k.rsplit(".", 1)[-1]
            if leaf in ("beta", "gamma"):
                v = torch.zeros(e.ref_shape)
            elif ".norm" in k:
                v = torch.ones(e.ref_shape) if leaf == "weight" else torch.zeros(e.ref_shape)
            elif leaf == "weight":
                fan_in = e.ref_shape[1] * e.ref_shape[2] * e.ref_shape[3]
                bound = 1.0 / fan_in ** 0.5
                v = torch.empty(e.ref_shape).uniform_(-bound, bound)
            else:  # bias: fan_in of the owning conv
                wk = k[:-4] + "weight"
                ws = self.entries[wk].ref_shape
                bound = 1.0 / (ws[1] * ws[2] * ws[3]) ** 0.5
                v = torch.empty(e.ref_shape).uniform_(-bound, bound)
            self.flat.data[e.offset:e.offset + e.numel] = self._to_internal(e, v)

    # ------------------------------------------------------------------ state dict in reference form
    def _save_to_state_dict(self, destination, prefix, keep_vars):
        flat = self.flat if keep_vars else self.flat.detach()
        for k in self.ref_order:
            e = self.entries[k]
            destination[prefix + k] = self._to_reference(e, flat[e.offset:e.offset + e.numel])

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        seen = set()
        with torch.no_grad():
            for k in self.ref_order:
                e = self.entries[k]
                full = prefix + k
                if full not in state_dict:
                    missing_keys.append(full)
                    continue
                v = state_dict[full]
                if tuple(v.shape) != e.ref_shape:
                    error_msgs.append(f"size mismatch for {full}: copying {tuple(v.shape)}, expected {e.ref_shape}")
                    continue
                self.flat.data[e.offset:e.offset + e.numel] = self._to_internal(e, v.to(self.flat.device,
                                                                                        torch.float32))
                seen.add(full)
        if strict:
            for k in state_dict:
                if k.startswith(prefix) and k not in seen and k[len(prefix):] not in self.entries:
                    unexpected_keys.append(k)

    # ------------------------------------------------------------------ forward
    def check_image_size_hw(self, h: int, w: int) -> Tuple[int, int]:
        ps = self.padder_size
        return h + (ps - h % ps) % ps, w + (ps - w % ps) % ps

    def forward(self, inp: torch.Tensor) -> torch.Tensor:
        _lib.require_cuda(inp)
        if inp.dim() != 4 or inp.shape[1] != self.img_channel:
            raise ValueError(f"expected [B,{self.img_channel},H,W], got {tuple(inp.shape)}")
        inp = inp.contiguous()
        if torch.is_grad_enabled() and (self.flat.requires_grad or inp.requires_grad):
            return _NAFNetFn.apply(inp, self.flat, self)
        out, _ = self.exec_forward(inp, save=False)
        return out

    # The executor.  Every op appends a record to the tape when save=True.
    def exec_forward(self, x: torch.Tensor, save: bool, flat: Optional[torch.Tensor] = None):
        P = self.flat.data if flat is None else flat
        B, Ci, H0, W0 = x.shape
        Hp, Wp = self.check_image_size_hw(H0, W0)
        tape: List[tuple] = []
        Wt = (P,) if self.precision == "fp32" else (P,) + self._prep_weights(P)
        self._W = Wt
        self._ln_carry = None
        w = self.width
        feat = torch.empty(B, Hp, Wp, w, device=x.device, dtype=self.adt)
        call("intro_fwd", x, self._slice(P, "intro.weight"), self._slice(P, "intro.bias"), feat, B, Ci, H0, W0, Hp,
             Wp, w, self.dt)
        if save:
            tape.append(("intro", x, (B, Ci, H0, W0, Hp, Wp, w)))
        h, wd = Hp, Wp
        skips = []
        for i, n in enumerate(self.enc_blk_nums):
            c = self.enc_chans[i]
            for j in range(n):
                nxt = f"encoders.{i}.{j + 1}." if j + 1 < n else None
                feat = self._block_fwd(P, f"encoders.{i}.{j}.", feat, B, h, wd, c, tape if save else None, nxt)
            skips.append(feat)
            feat = self._down_fwd(P, i, feat, B, h, wd, c, tape if save else None)
            h, wd = h // 2, wd // 2
        for j in range(self.middle_blk_num):
            nxt = f"middle_blks.{j + 1}." if j + 1 < self.middle_blk_num else None
            feat = self._block_fwd(P, f"middle_blks.{j}.", feat, B, h, wd, self.mid_chan, tape if save else None, nxt)
        for i, n in enumerate(self.dec_blk_nums):
            chan = self.dec_chans[i] * 2
            feat = self._up_fwd(P, i, feat, skips[::-1][i], B, h, wd, chan, tape if save else None)
            h, wd = h * 2, wd * 2
            c = self.dec_chans[i]
            for j in range(n):
                nxt = f"decoders.{i}.{j + 1}." if j + 1 < n else None
                feat = self._block_fwd(P, f"decoders.{i}.{j}.", feat, B, h, wd, c, tape if save else None, nxt)
        out = torch.empty(B, Ci, H0, W0, device=x.device)
        call("ending_fwd", feat, self._slice(P, "ending.weight"), self._slice(P, "ending.bias"), x, out, B, Ci, H0,
             W0, Hp, Wp, w, self.dt)
        if save:
            tape.append(("ending", feat, (B, Ci, H0, W0, Hp, Wp, w)))
            tape.append(("weights", Wt))
        self._W = None
        return out, tape

    def _block_fwd(self, P, pre, x, B, h, w, c, tape, next_pre=None):
        """One NAFBlock forward (NAFNet_arch.py:60-80).  At C in {32, 64, 128} (bf16) the LayerNorms run in the epilogue
        of the GEMM producing their input (nbp_gemm_res_ln): norm2 in conv3's, the next block's norm1 (next_pre)
        in conv5's; that block then takes (n1, st1) from self._ln_carry."""
        M = B * h * w
        dev = x.device
        E = lambda *s: torch.empty(*s, device=dev, dtype=self.adt)  # noqa: E731
        F = lambda *s: torch.empty(*s, device=dev)  # noqa: E731  (fp32 statistics)
        dt = self.dt
        fuse_ln = self.fuse_ln_fwd and dt != 0 and len(self._W) >= 3 and c in (32, 64, 128, 256)
        carry, self._ln_carry = self._ln_carry, None
        have_n1 = carry is not None and carry[0] is x
        n1, st1 = (carry[1], carry[2]) if have_n1 else (E(M, c), F(M, 2))
        tile = len(self._W) >= 3 and self.tile_level(B, h, w, c)
        c1dw = (not tile and self.fuse_c1dw and dt != 0 and len(self._W) >= 3
                and query("c1dw_supported", h, w, c, dt) == 1)
        chunks = (query("c1dw_tile_rows", h, w, c) if tile else
                  (1 if c1dw else query("dw_fwd_slab_rows", B, h, w, c, dt)))
        # the tile path keeps no t1 / t2 (the backward rebuilds them from n1); t2 is dropped anyway without a tape
        t1 = None if tile else E(M, 2 * c)
        t2 = None if tile else E(M, 2 * c)
        g, pool = E(M, c), F(B * chunks * c)
        mean, a = F(B, c), F(B, c)
        y, n2, st2 = E(M, c), E(M, c), F(M, 2)
        # t4 channel pairs interleaved (conv4 rows stored so); at C = 32 it is dropped when the backward rebuilds
        # it (sg_rc) or there is no backward
        drop_t4 = dt != 0 and c == 32 and (tape is None or (self.sg_rc and self.fold_ls and len(self._W) >= 3))
        # the fused FFN half (g2 never stored) wherever the backward rebuilds g2 too (nbp_dgrad_sg_rc_wg)
        ffn = drop_t4 and self.fuse_ffn and len(self._W) >= 3 and (tape is None or self.sg_rc_wg)
        t4, g2 = (None if drop_t4 else E(M, 2 * c)), (None if ffn else E(M, c))
        out = E(M, c)
        hw = h * w
        # deep levels (C 128 / 256 / 512): conv3 -> norm2 -> conv4 -> SimpleGate -> conv5 (-> the next norm1) as ONE
        # row-stationary launch (nbp_ffn_rows_fwd, bitwise the launches it replaces)
        rows_ffn = (self.fuse_ffn_rows and dt != 0 and len(self._W) >= 4 and self._W[3] is not None and t4 is not None
                    and g2 is not None and query("ffn_rows_supported", M, c, hw, dt) == 1)
        carry_next = (fuse_ln or rows_ffn) and next_pre is not None
        nn1, nst1 = (E(M, c), F(M, 2)) if carry_next else (None, None)
        if not have_n1:
            call("ln_fwd_nhwc", x, self._slice(P, pre + "norm1.weight"), self._slice(P, pre + "norm1.bias"),
                 n1, st1, M, c, LN_EPS, dt)
        if tile:
            call("c1dw_fwd_tile", n1, self._slice(self._W[1], pre + "conv1.weight"), self._slice(P, pre + "conv1.bias"),
                 self._slice(P, pre + "conv2.weight"), self._slice(P, pre + "conv2.bias"), None, None, g, pool, B, h, w,
                 c, dt)
        elif c1dw:
            call("c1_dw_sg_pool", n1, self._slice(self._W[1], pre + "conv1.weight"), self._slice(P, pre + "conv1.bias"),
                 self._slice(P, pre + "conv2.weight"), self._slice(P, pre + "conv2.bias"), t1, t2, g, pool, B, h, w,
                 c, dt)
        else:
            self._mm(self._W, n1, c, AM_PLAIN, None, 1, pre + "conv1.weight", t1, 2 * c, CM_PLAIN, M, 2 * c,
                     c, bias=self._slice(P, pre + "conv1.bias"))
            call("dw_sg_pool_fwd", t1, self._slice(P, pre + "conv2.weight"), self._slice(P, pre + "conv2.bias"),
                 t2, g, pool, B, h, w, c, dt)
        call("sca_fwd", pool, chunks, self._slice(P, pre + "sca.1.weight"), self._slice(P, pre + "sca.1.bias"),
             mean, a, B, hw, c)
        if rows_ffn:
            lnw, lnb = ((self._slice(P, next_pre + "norm1.weight"), self._slice(P, next_pre + "norm1.bias"))
                        if carry_next else (None, None))
            call("ffn_rows_fwd", g, a, hw, x, self._slice(self._W[3], pre + "conv3.weight"),
                 self._slice(P, pre + "conv3.bias"), self._slice(P, pre + "beta"), self._slice(P, pre + "norm2.weight"),
                 self._slice(P, pre + "norm2.bias"), self._slice(self._W[3], pre + "conv4.weight"),
                 self._slice(P, pre + "conv4.bias"), self._slice(self._W[3], pre + "conv5.weight"),
                 self._slice(P, pre + "conv5.bias"), self._slice(P, pre + "gamma"), lnw, lnb, y, n2, st2, t4, g2, out,
                 nn1, nst1, M, c, LN_EPS, dt)
        elif fuse_ln:
            call("gemm_res_ln", g, c, AM_SCALE, a, hw, self._slice(self._W[1], pre + "conv3.weight"), c, y,
                 M, c, c, self._slice(P, pre + "conv3.bias"), x, self._slice(P, pre + "beta"),
                 self._slice(P, pre + "norm2.weight"), self._slice(P, pre + "norm2.bias"), n2, st2, LN_EPS,
                 dt)
        else:
            self._mm(self._W, g, c, AM_SCALE, a, hw, pre + "conv3.weight", y, c, CM_PLAIN, M, c, c,
                     bias=self._slice(P, pre + "conv3.bias"), R=x, rscale=self._slice(P, pre + "beta"))
            call("ln_fwd_nhwc", y, self._slice(P, pre + "norm2.weight"), self._slice(P, pre + "norm2.bias"),
                 n2, st2, M, c, LN_EPS, dt)
        if rows_ffn:
            pass
        elif ffn:
            lnw, lnb = ((self._slice(P, next_pre + "norm1.weight"), self._slice(P, next_pre + "norm1.bias"))
                        if carry_next else (None, None))
            call("gemm_ffn", n2, self._slice(self._W[1], pre + "conv4.weight"), self._slice(P, pre + "conv4.bias"),
                 self._slice(self._W[1], pre + "conv5.weight"), self._slice(P, pre + "conv5.bias"), y,
                 self._slice(P, pre + "gamma"), lnw, lnb, out, nn1, nst1, M, c, LN_EPS, dt)
        elif dt != 0:  # SimpleGate in the GEMM epilogue
            self._mm(self._W, n2, c, AM_PLAIN, None, 1, pre + "conv4.weight", t4, 2 * c, CM_SG, M, 2 * c, c,
                     bias=self._slice(P, pre + "conv4.bias"), pre=g2)
        else:
            self._mm(self._W, n2, c, AM_PLAIN, None, 1, pre + "conv4.weight", t4, 2 * c, CM_PLAIN, M, 2 * c,
                     c, bias=self._slice(P, pre + "conv4.bias"))
            call("sg_fwd", t4, g2, M, c, 1, dt)
        if ffn or rows_ffn:
            pass
        elif carry_next:
            call("gemm_res_ln", g2, c, AM_PLAIN, None, 1, self._slice(self._W[1], pre + "conv5.weight"), c,
                 out, M, c, c, self._slice(P, pre + "conv5.bias"), y, self._slice(P, pre + "gamma"),
                 self._slice(P, next_pre + "norm1.weight"), self._slice(P, next_pre + "norm1.bias"), nn1,
                 nst1, LN_EPS, dt)
        else:
            self._mm(self._W, g2, c, AM_PLAIN, None, 1, pre + "conv5.weight", out, c, CM_PLAIN, M, c, c,
                     bias=self._slice(P, pre + "conv5.bias"), R=y, rscale=self._slice(P, pre + "gamma"))

        if carry_next:
            self._ln_carry = (out.view(B, h, w, c), nn1, nst1)
        if tape is not None:
            tape.append(("block", pre, (B, h, w, c), dict(x=x, n1=n1, st1=st1, t1=t1, t2=t2, g=g, mean=mean, a=a, y=y,
                                                           n2=n2, st2=st2, t4=t4, g2=g2)))
        return self._ln_carry[0] if self._ln_carry is not None else out.view(B, h, w, c)

    def tile_level(self, B: int, h: int, w: int, c: int) -> bool:
        """Whether a block of this level takes the tile path (nbp_c1dw_fwd_tile / nbp_c1dw_bwd_tile: t1 / t2 rebuilt on
        chip): 16-bit modes, the channel counts in c1dw_tile_channels, and a level small enough for the kernels' 32-bit
        buffer offsets (nbp_c1dw_tile_supported depends on B: e.g. 16 images of 1024^2 at level 0 take the stored
        tape)."""
        dt = self.dt
        return (self.fuse_c1dw_tile and c in self.c1dw_tile_channels and dt != 0
                and query("c1dw_tile_supported", B, h, w, c, dt) == 1)

    def _down_fwd(self, P, i, x, B, h, w, c, tape):
        ho, wo = h // 2, w // 2
        M = B * ho * wo
        out = torch.empty(B, ho, wo, 2 * c, device=x.device, dtype=self.adt)
        self._mm(self._W, x, 0, AM_S2D, None, 1, f"downs.{i}.weight", out, 2 * c, CM_PLAIN, M, 2 * c, 4 * c, ho, wo,
                 c, bias=self._slice(P, f"downs.{i}.bias"))
        if tape is not None:
            tape.append(("down", i, (B, h, w, c), x))
        return out

    def _up_fwd(self, P, i, x, skip, B, h, w, chan, tape):
        M = B * h * w
        out = torch.empty(B, 2 * h, 2 * w, chan // 2, device=x.device, dtype=self.adt)
        self._mm(self._W, x, chan, AM_PLAIN, None, 1, f"ups.{i}.0.weight", out, 0, CM_D2S, M, 2 * chan, chan, h, w,
                 chan // 2, R=skip)
        if tape is not None:
            tape.append(("up", i, (B, h, w, chan), x))
        return out

    # ------------------------------------------------------------------ backward
    def exec_backward(self, tape, dout: torch.Tensor, dflat: torch.Tensor, need_dx: bool,
                      flat: Optional[torch.Tensor] = None, hook: Optional[Callable[[Stage], None]] = None):
        """Walk the tape in reverse.  Writes every parameter gradient (exactly once) into dflat, calls
        hook(stage) as each stage's gradient slice is complete, returns d(input) or None."""
        P = self.flat.data if flat is None else flat
        self._keep = []
        call("grad_reduce_defer")
        try:
            return self._walk_backward(tape, dout, dflat, need_dx, P, hook)
        finally:
            if self._grouping:  # an error inside a grouped level: launch what is queued so the library state is reset
                self._grouping = False
                call("wgrad_group", 0)
            call("grad_reduce_flush", 1)
            self._keep = None

    def _level_grouped(self, c: int) -> bool:
        return self.dt != 0 and c % 128 == 0 and self.group_wgrad

    def _close_level(self, pending: List[str], hook):
        """Launch the level's queued weight gradients, then complete its stages (flush + DP hooks) in order."""
        self._grouping = False
        call("wgrad_group", 0)
        for name in pending:
            self._stage_done(name, hook)

    def _walk_backward(self, tape, dout, dflat, need_dx, P, hook):
        Wt = (P,)
        for rec in tape:
            if rec[0] == "weights":
                Wt = rec[1]
        dfeat = None
        dskips: List[torch.Tensor] = []
        dx_img = None
        level: Optional[List[str]] = None  # stages of the current grouped level, completed when it closes
        level_c = 0
        pend = None  # a block's deferred conv1 input gradient + norm1 backward (taken by the preceding block)
        recs = [r for r in reversed(tape) if r[0] != "weights"]
        for idx, rec in enumerate(recs):
            kind = rec[0]
            if pend is not None and kind != "block":  # not expected (deferral looks ahead to a block): resolve it
                dfeat, pend = self._conv1_bwd(P, Wt, dflat, **pend), None
            grouped = kind == "block" and self._level_grouped(rec[2][3])
            if level is not None and not (grouped and rec[2][3] == level_c):
                self._close_level(level, hook)
                level = None
            if grouped and level is None:
                call("wgrad_group", 1)
                self._grouping = True
                level, level_c = [], rec[2][3]
            if kind == "ending":
                feat, (B, Ci, H0, W0, Hp, Wp, w) = rec[1], rec[2]
                dfeat = torch.empty(B, Hp, Wp, w, device=dout.device, dtype=self.adt)
                ws = self._ws(query("ending_bwd_workspace_floats", B, Ci, H0, W0, w), dout.device)
                call("ending_bwd", dout, feat, self._slice(P, "ending.weight"), dfeat,
                     self._slice(dflat, "ending.weight"), self._slice(dflat, "ending.bias"), ws, B, Ci, H0, W0, Hp,
                     Wp, w, self.dt)
                self._stage_done("ending", hook)
            elif kind == "block":
                pre, geo, S = rec[1], rec[2], rec[3]
                # defer into the preceding block of the same (grouped) level when that one takes the row-stationary
                # backward: the norm1 gradients of this block then land before the level closes
                nxt = recs[idx + 1] if idx + 1 < len(recs) else None
                defer = (self.ffn_rows_pre and level is not None and nxt is not None and nxt[0] == "block"
                         and tuple(nxt[2]) == tuple(geo) and self._rows_ok(Wt, nxt[3], geo))
                dfeat, pend = self._block_bwd(P, Wt, dflat, pre, geo, S, dfeat, pend, defer)
                if level is not None:
                    level.append(pre[:-1])
                else:
                    self._stage_done(pre[:-1], hook)
            elif kind == "up":
                i, (B, h, w, chan), x = rec[1], rec[2], rec[3]
                dskips.append(dfeat)  # d(skip) = d(up output): the skip add is an identity branch
                M = B * h * w
                dx = torch.empty(B, h, w, chan, device=dout.device, dtype=self.adt)
                self._mm(Wt, dfeat, 0, AM_S2D, None, 1, f"ups.{i}.0.weight", dx, chan, CM_PLAIN, M, chan, 2 * chan,
                         h, w, chan // 2, dgrad=True)
                self._wgrad(dfeat, 0, AM_S2D, x, chan, AM_PLAIN, None, 1, M, 2 * chan, chan, h, w, chan // 2, 0,
                            self._slice(dflat, f"ups.{i}.0.weight"), None)
                self._stage_done(f"ups.{i}", hook)
                dfeat = dx
            elif kind == "down":
                i, (B, h, w, c), x = rec[1], rec[2], rec[3]
                ho, wo = h // 2, w // 2
                M = B * ho * wo
                dskip = dskips.pop()
                dx = torch.empty(B, h, w, c, device=dout.device, dtype=self.adt)
                # d enc = D2S(dout . Wd) + d skip
                self._mm(Wt, dfeat, 2 * c, AM_PLAIN, None, 1, f"downs.{i}.weight", dx, 0, CM_D2S, M, 4 * c, 2 * c,
                         ho, wo, c, R=dskip, dgrad=True)
                self._wgrad(dfeat, 2 * c, AM_PLAIN, x, 0, AM_S2D, None, 1, M, 2 * c, 4 * c, ho, wo, 0, c,
                            self._slice(dflat, f"downs.{i}.weight"), self._slice(dflat, f"downs.{i}.bias"))
                self._stage_done(f"downs.{i}", hook)
                dfeat = dx
            elif kind == "intro":
                x, (B, Ci, H0, W0, Hp, Wp, w) = rec[1], rec[2]
                ws = self._ws(query("intro_bwd_workspace_floats", B, Ci, Hp, Wp, w), dout.device)
                if need_dx:
                    dx_img = torch.empty(B, Ci, H0, W0, device=dout.device)
                call("intro_bwd", x, dfeat, self._slice(P, "intro.weight"), self._slice(dflat, "intro.weight"),
                     self._slice(dflat, "intro.bias"), dx_img, ws, B, Ci, H0, W0, Hp, Wp, w, self.dt)
                self._stage_done("intro", hook)
        if level is not None:
            self._close_level(level, hook)
        if need_dx:
            # global residual x + inp (NAFNet_arch.py:153): d inp += d out
            call("add", dx_img, dout, dx_img, dx_img.numel(), 0)
        return dx_img

    def _stage_done(self, name, hook):
        # the stage's queued gradient reductions run before anyone (the DP all-reduce hook) reads its slice; without a
        # hook they all wait for the backward's final flush (_LATE_FLUSH)
        if hook is None and _LATE_FLUSH:
            return
        call("grad_reduce_flush", 0)
        self._keep.clear()
        if hook is not None:
            hook(self.stages[name])

    def _ws(self, n, dev):
        """fp32 workspace that stays referenced until the next gradient-reduction flush (deferred reductions read
        it after this call returns)."""
        t = torch.empty(n, device=dev)
        if self._keep is not None:
            self._keep.append(t)
        return t

    def _wgrad(self, G, ldg, gmode, X, ldx, xmode, xscale, rows, M, N, K, gh, gw, csg, csx, dW, db, dtype=None):
        """Weight gradient (its output only feeds the stage's deferred reductions)."""
        n_ws = query("wgrad_workspace_floats", M, N, K)
        ws = self._ws(n_ws, G.device)
        if self._grouping and self._keep is not None:  # the launch is deferred to the level's end: keep the operands
            self._keep.extend(t for t in (G, X, xscale) if t is not None)
        call("wgrad_f32", G, ldg, gmode, X, ldx, xmode, xscale, rows, M, N, K, gh, gw, csg, csx, dW, db, ws,
             n_ws, self.dt if dtype is None else dtype)

    def _reduce(self, slab, S, L, out):
        call("reduce_slab", slab, S, L, out)

    def _ffn_bwd_launches(self, P, Wt, dflat, pre, B, h, w, c, S, dout):
        """The FFN half's backward as separate launches; returns (dy, dh, SCA channel-dot slab, its chunks per image)."""
        M = B * h * w
        HW = h * w
        dev = dout.device
        E = lambda *s: torch.empty(*s, device=dev, dtype=self.adt)  # noqa: E731
        F = lambda *s: self._ws(math.prod(s), dev)  # noqa: E731  (slabs live until the stage's flush)
        dt = self.dt
        # out = y + gamma * conv5(g2): no stored pre-activation, no scaled-gradient pass.  dg2 = (gamma (.) dout) W5
        # (gamma as the A-operand column scale); U5 = dout^T g2, V5 = colsum dout feed dW5 = gamma (.) U5,
        # db5 = gamma (.) V5, dgamma = rowsum(W5 (.) U5) + b5 (.) V5 (nbp_layer_scale_grad, after the reductions).
        dt4 = E(M, 2 * c)
        folded = len(Wt) >= 3 and self.fold_ls  # gamma / beta already in the transposed bf16 weights
        U5, V5 = F(c * c), F(c)
        wg_folded = False
        if dt != 0:  # SimpleGate backward in the dgrad epilogue: dg2 never materialises
            if S["t4"] is None:  # t4 = conv4(n2) rebuilt per tile inside the dgrad (level 0, folded layer scale)
                assert folded and c == 32
                args = (dout, c, self._slice(Wt[2], pre + "conv5.weight"), c, S["n2"],
                        self._slice(Wt[1], pre + "conv4.weight"), self._slice(P, pre + "conv4.bias"), dt4, M, c, c)
                if self.sg_rc_wg:  # + U5 / V5 and conv4's dW / db from the same tiles
                    n_ws = query("dgrad_sg_rc_wg_workspace_floats", M, c)
                    call("dgrad_sg_rc_wg", *args, U5, V5, self._slice(dflat, pre + "conv4.weight"),
                         self._slice(dflat, pre + "conv4.bias"), F(n_ws), n_ws, dt)
                    wg_folded = True
                else:
                    call("dgrad_sg_rc", *args, dt)
            elif folded:
                self._mm(Wt, dout, c, AM_PLAIN, None, 1, pre + "conv5.weight", dt4, 2 * c, CM_SGBWD, M, c, c,
                         R=S["t4"], dgrad=True)
            else:
                self._mm(Wt, dout, c, AM_SCALE, self._slice(P, pre + "gamma"), M, pre + "conv5.weight", dt4, 2 * c,
                         CM_SGBWD, M, c, c, R=S["t4"], dgrad=True)
        else:
            dg2 = E(M, c)
            self._mm(Wt, dout, c, AM_SCALE, self._slice(P, pre + "gamma"), M, pre + "conv5.weight", dg2, c, CM_PLAIN,
                     M, c, c, dgrad=True)
            call("sg_bwd", dg2, S["t4"], dt4, M, c, 1, dt)
        # at C >= 128 the wide weight gradients below are queued into the level's grouped launch (_walk_backward)
        if not wg_folded:
            self._wgrad(dout, c, AM_PLAIN, S["g2"], c, AM_PLAIN, None, 1, M, c, c, 0, 0, 0, 0, U5, V5)
        call("layer_scale_grad", U5, V5, self._slice(P, pre + "conv5.weight"), self._slice(P, pre + "conv5.bias"),
             self._slice(P, pre + "gamma"), self._slice(dflat, pre + "conv5.weight"),
             self._slice(dflat, pre + "conv5.bias"), self._slice(dflat, pre + "gamma"), c, c)
        # conv4 input gradient + norm2 backward + residual
        # LN backward in the dgrad's epilogue (dn never stored): skinny kernel at C 32 / 64, 64 x 128 tiles at 128
        fuse_ln = dt != 0 and c in (32, 64, 128, 256)
        dy = E(M, c)
        if not wg_folded:
            self._wgrad(dt4, 2 * c, AM_PLAIN, S["n2"], c, AM_PLAIN, None, 1, M, 2 * c, c, 0, 0, 0, 0,
                        self._slice(dflat, pre + "conv4.weight"), self._slice(dflat, pre + "conv4.bias"))
        if fuse_ln:
            self._dgrad_ln(Wt, dflat, P, pre, "conv4.weight", "norm2", dt4, S["y"].reshape(M, c), S["st2"], dout, dy,
                           M, c)
        else:
            dn2 = E(M, c)
            self._mm(Wt, dt4, 2 * c, AM_PLAIN, None, 1, pre + "conv4.weight", dn2, c, CM_PLAIN, M, c, 2 * c,
                     dgrad=True)
            lg = query("ln_nhwc_grid", M, c, dt)
            sw, sb = F(lg * c), F(lg * c)
            call("ln_bwd_nhwc", dn2, S["y"].reshape(M, c), S["st2"], self._slice(P, pre + "norm2.weight"), dout, dy,
                 sw, sb, M, c, dt)
            self._reduce(sw, lg, c, self._slice(dflat, pre + "norm2.weight"))
            self._reduce(sb, lg, c, self._slice(dflat, pre + "norm2.bias"))
        # y = x + beta * conv3(h), h = g (.) a: same layer-scale identity as conv5 (dh = (beta (.) dy) W3)
        dh = E(M, c)
        # tiled-GEMM levels (C > 64): the SCA channel dot sum_p dh (.) g rides in the dgrad epilogue (CM_CHANDOT,
        # per-64-row-tile partials); levels 0/1 (skinny GEMM) keep img_chan_dot
        chandot = folded and c > 64 and HW % 64 == 0
        if chandot:
            chunks = HW // 64
            da_slab = F(B * chunks * c)
            call("gemm_bf16", dy, c, AM_PLAIN, None, HW, dt, self._slice(Wt[2], pre + "conv3.weight"), c, dh, c,
                 CM_CHANDOT, dt, M, c, c, 0, 0, 0, None, S["g"], None, da_slab)
        elif folded:
            self._mm(Wt, dy, c, AM_PLAIN, None, 1, pre + "conv3.weight", dh, c, CM_PLAIN, M, c, c, dgrad=True)
        else:
            self._mm(Wt, dy, c, AM_SCALE, self._slice(P, pre + "beta"), M, pre + "conv3.weight", dh, c, CM_PLAIN, M,
                     c, c, dgrad=True)
        U3, V3 = F(c * c), F(c)
        self._wgrad(dy, c, AM_PLAIN, S["g"], c, AM_SCALE, S["a"], HW, M, c, c, 0, 0, 0, 0, U3, V3)
        call("layer_scale_grad", U3, V3, self._slice(P, pre + "conv3.weight"), self._slice(P, pre + "conv3.bias"),
             self._slice(P, pre + "beta"), self._slice(dflat, pre + "conv3.weight"),
             self._slice(dflat, pre + "conv3.bias"), self._slice(dflat, pre + "beta"), c, c)
        # SCA
        if not chandot:
            chunks = query("dw_chunks", B, h, w, c, 0)
            da_slab = F(B * chunks * c)
            call("img_chan_dot", dh, S["g"], da_slab, B, h, w, c, dt)
        return dy, dh, da_slab, chunks

    def _rows_ok(self, Wt, S, geo) -> bool:
        """Whether a block's FFN backward takes the row-stationary launch (nbp_ffn_rows_bwd)."""
        B, h, w, c = geo
        return (self.fuse_ffn_rows and self.dt != 0 and len(Wt) >= 5 and Wt[4] is not None and self.fold_ls
                and S["t4"] is not None and S["g2"] is not None
                and query("ffn_rows_supported", B * h * w, c, h * w, self.dt) == 1)

    def _ffn_bwd_rows(self, P, Wt, dflat, pre, B, h, w, c, S, dout, pend=None):
        """The FFN half's backward in one row-stationary launch (nbp_ffn_rows_bwd: dt4, dy, dh bitwise the launches; the
        norm2 weight / bias and SCA channel-dot partials per 32-row block), then the weight gradients it feeds queued
        as in _ffn_bwd_launches.  With pend (the following block's deferred conv1 input gradient, dout None) the launch
        first makes that block's dx = this block's dout (bitwise _conv1_bwd), its norm1 partials reduced here.  Returns
        (dy, dh, SCA slab, chunks per image, dout)."""
        M = B * h * w
        HW = h * w
        dev = (dout if dout is not None else pend["dt1"]).device
        E = lambda *s: torch.empty(*s, device=dev, dtype=self.adt)  # noqa: E731
        F = lambda *s: self._ws(math.prod(s), dev)  # noqa: E731  (slabs live until the stage's flush)
        dt = self.dt
        nb = M // 32
        dt4, dy, dh = E(M, 2 * c), E(M, c), E(M, c)
        sw, sb, da_slab = F(nb * c), F(nb * c), F(nb * c)
        pre_args = (None,) * 9
        if pend is not None:
            q = pend["pre"]
            dout = E(M, c)
            sw1, sb1 = F(nb * c), F(nb * c)
            pre_args = (pend["dt1"], self._slice(Wt[4], q + "conv1.weight"), pend["x"], pend["st1"],
                        self._slice(P, q + "norm1.weight"), pend["dy"], dout, sw1, sb1)
        call("ffn_rows_bwd", None if pend is not None else dout, S["t4"], S["y"].reshape(M, c), S["st2"],
             self._slice(P, pre + "norm2.weight"), S["g"], self._slice(Wt[4], pre + "conv5.weight"),
             self._slice(Wt[4], pre + "conv4.weight"), self._slice(Wt[4], pre + "conv3.weight"), dt4, dy, dh, sw, sb,
             da_slab, *pre_args, M, c, HW, dt)
        if pend is not None:
            self._reduce(sw1, nb, c, self._slice(dflat, pend["pre"] + "norm1.weight"))
            self._reduce(sb1, nb, c, self._slice(dflat, pend["pre"] + "norm1.bias"))
        U5, V5 = F(c * c), F(c)
        self._wgrad(dout, c, AM_PLAIN, S["g2"], c, AM_PLAIN, None, 1, M, c, c, 0, 0, 0, 0, U5, V5)
        call("layer_scale_grad", U5, V5, self._slice(P, pre + "conv5.weight"), self._slice(P, pre + "conv5.bias"),
             self._slice(P, pre + "gamma"), self._slice(dflat, pre + "conv5.weight"),
             self._slice(dflat, pre + "conv5.bias"), self._slice(dflat, pre + "gamma"), c, c)
        self._wgrad(dt4, 2 * c, AM_PLAIN, S["n2"], c, AM_PLAIN, None, 1, M, 2 * c, c, 0, 0, 0, 0,
                    self._slice(dflat, pre + "conv4.weight"), self._slice(dflat, pre + "conv4.bias"))
        self._reduce(sw, nb, c, self._slice(dflat, pre + "norm2.weight"))
        self._reduce(sb, nb, c, self._slice(dflat, pre + "norm2.bias"))
        U3, V3 = F(c * c), F(c)
        self._wgrad(dy, c, AM_PLAIN, S["g"], c, AM_SCALE, S["a"], HW, M, c, c, 0, 0, 0, 0, U3, V3)
        call("layer_scale_grad", U3, V3, self._slice(P, pre + "conv3.weight"), self._slice(P, pre + "conv3.bias"),
             self._slice(P, pre + "beta"), self._slice(dflat, pre + "conv3.weight"),
             self._slice(dflat, pre + "conv3.bias"), self._slice(dflat, pre + "beta"), c, c)
        return dy, dh, da_slab, HW // 32, dout

    def _block_bwd(self, P, Wt, dflat, pre, geo, S, dout, pend=None, defer=False):
        """One block's backward.  dout None: the following block's conv1 input gradient is pending (pend) and made by
        this block's row-stationary launch.  defer: this block's own conv1 input gradient + norm1 backward is left
        pending for the preceding block.  Returns (dx or None, pending or None)."""
        B, h, w, c = geo
        M = B * h * w
        HW = h * w
        dt = self.dt
        # the FFN half's backward: conv5 dgrad + SimpleGate backward, conv4 dgrad + norm2 backward, conv3 dgrad (+ the SCA
        # channel-dot partials) and the weight gradients they feed
        rows = self._rows_ok(Wt, S, geo)
        if pend is not None and not rows:  # not expected (the walker's look-ahead uses the same test): resolve it here
            dout, pend = self._conv1_bwd(P, Wt, dflat, **pend), None
        if rows:
            dy, dh, da_slab, chunks, dout = self._ffn_bwd_rows(P, Wt, dflat, pre, B, h, w, c, S,
                                                               None if pend is not None else dout.reshape(M, c), pend)
        else:
            dout = dout.reshape(M, c)
            dy, dh, da_slab, chunks = self._ffn_bwd_launches(P, Wt, dflat, pre, B, h, w, c, S, dout)
        dev = dout.device
        E = lambda *s: torch.empty(*s, device=dev, dtype=self.adt)  # noqa: E731
        F = lambda *s: self._ws(math.prod(s), dev)  # noqa: E731  (slabs live until the stage's flush)
        # ds = da . W_sca and the SCA weight gradients dW = da^T mean, db = colsum(da) in one launch (or inside the
        # depthwise backward below)
        env = __import__("os").environ
        sca_fold = self.sca_fold and dt != 0 and c <= 1024 and B <= 256 and (
            (S["t1"] is not None and c % 16 == 0)  # nbp_sca_dw_bwd
            or (S["t1"] is None and not env.get("NBP_C1DW_BWD_TH") and not env.get("NBP_C1DW_BWD_BAL")))  # the tile
        if not sca_fold:
            ds = F(B, c)
            call("sca_bwd_fused", da_slab, chunks, self._slice(P, pre + "sca.1.weight"), S["mean"], ds,
                 self._slice(dflat, pre + "sca.1.weight"), self._slice(dflat, pre + "sca.1.bias"), B, c)
        # SimpleGate + depthwise conv2 (fused when the channel slicing allows: dt2 stays in LDS)
        dt1 = E(M, 2 * c)
        if S["t1"] is None:  # levels 0 / 1 tile path: t1 / t2 rebuilt from n1 on chip (nbp_c1dw_bwd_tile)
            ws = F(query("c1dw_bwd_workspace_floats", B, h, w, c))
            tail = (S["n1"], self._slice(Wt[1], pre + "conv1.weight"), self._slice(P, pre + "conv1.bias"),
                    self._slice(P, pre + "conv2.weight"), self._slice(P, pre + "conv2.bias"), dt1,
                    self._slice(dflat, pre + "conv2.weight"), self._slice(dflat, pre + "conv2.bias"), ws, B, h, w, c, dt)
            if sca_fold:
                call("sca_c1dw_bwd_tile", dh, S["a"], da_slab, chunks, self._slice(P, pre + "sca.1.weight"), S["mean"],
                     self._slice(dflat, pre + "sca.1.weight"), self._slice(dflat, pre + "sca.1.bias"), *tail)
            else:
                call("c1dw_bwd_tile", dh, S["a"], ds, *tail)
        else:
            ws = F(query("dw_bwd_workspace_floats", B, h, w, c))
            dw_args = (S["t1"], self._slice(P, pre + "conv2.weight"), dt1, self._slice(dflat, pre + "conv2.weight"),
                       self._slice(dflat, pre + "conv2.bias"), ws, B, h, w, c, dt)
        if sca_fold and S["t1"] is not None:
            call("sca_dw_bwd", dh, S["a"], da_slab, chunks, self._slice(P, pre + "sca.1.weight"), S["mean"],
                 self._slice(dflat, pre + "sca.1.weight"), self._slice(dflat, pre + "sca.1.bias"), S["t2"], *dw_args)
        elif S["t1"] is not None and c % (16 if dt != 0 else 8) == 0:
            call("sca_sg_dw_bwd", dh, S["a"], ds, S["t2"], *dw_args)
        elif S["t1"] is not None:
            dt2 = E(M, 2 * c)
            call("sca_sg_bwd", dh, S["a"], ds, S["t2"], dt2, M, c, HW, dt)
            call("dw_bwd", dt2, *dw_args)
        # conv1 input gradient + norm1 backward + residual
        if dt != 0 and c == 32 and self.ln_wg:  # + conv1's dW / db from the same tiles (n1 rebuilt from x / stats)
            dx = E(M, c)
            n_ws = query("dgrad_ln_bwd_wg_workspace_floats", M, c)
            call("dgrad_ln_bwd_wg", dt1, 2 * c, self._slice(Wt[2], pre + "conv1.weight"), 2 * c, M, c, 2 * c,
                 S["x"].reshape(M, c), S["st1"], self._slice(P, pre + "norm1.weight"),
                 self._slice(P, pre + "norm1.bias"), dy, dx, self._slice(dflat, pre + "norm1.weight"),
                 self._slice(dflat, pre + "norm1.bias"), self._slice(dflat, pre + "conv1.weight"),
                 self._slice(dflat, pre + "conv1.bias"), F(n_ws), n_ws, dt)
            return dx.view(B, h, w, c), None
        self._wgrad(dt1, 2 * c, AM_PLAIN, S["n1"], c, AM_PLAIN, None, 1, M, 2 * c, c, 0, 0, 0, 0,
                    self._slice(dflat, pre + "conv1.weight"), self._slice(dflat, pre + "conv1.bias"))
        pend = dict(pre=pre, geo=geo, dt1=dt1, x=S["x"].reshape(M, c), st1=S["st1"], dy=dy)
        if defer:
            return None, pend
        return self._conv1_bwd(P, Wt, dflat, **pend), None

    def _conv1_bwd(self, P, Wt, dflat, pre, geo, dt1, x, st1, dy):
        """conv1 input gradient + norm1 backward + the residual dy: a block's dx."""
        B, h, w, c = geo
        M = B * h * w
        dt = self.dt
        dx = torch.empty(M, c, device=dt1.device, dtype=self.adt)
        # LN backward in the conv1 dgrad's epilogue (dn1 never stored) at these widths
        if dt != 0 and c in (32, 64, 128, 256):
            self._dgrad_ln(Wt, dflat, P, pre, "conv1.weight", "norm1", dt1, x, st1, dy, dx, M, c)
        else:
            dn1 = torch.empty(M, c, device=dt1.device, dtype=self.adt)
            self._mm(Wt, dt1, 2 * c, AM_PLAIN, None, 1, pre + "conv1.weight", dn1, c, CM_PLAIN, M, c, 2 * c,
                     dgrad=True)
            lg = query("ln_nhwc_grid", M, c, dt)
            sw, sb = self._ws(lg * c, dt1.device), self._ws(lg * c, dt1.device)
            call("ln_bwd_nhwc", dn1, x, st1, self._slice(P, pre + "norm1.weight"), dy, dx, sw, sb, M, c, dt)
            self._reduce(sw, lg, c, self._slice(dflat, pre + "norm1.weight"))
            self._reduce(sb, lg, c, self._slice(dflat, pre + "norm1.bias"))
        return dx.view(B, h, w, c)

    def _dgrad_ln(self, Wt, dflat, P, pre, wkey, norm, dt, x, st, dres, out, M, c):
        """dn = dt . W (bf16 transposed weight copy) and the LayerNorm2d backward + residual in one launch
        (nbp_dgrad_ln_bwd); the LN weight / bias gradients are slab-reduced with the stage's deferred reductions."""
        n_ws = query("dgrad_ln_workspace_floats", M, c)
        ws = self._ws(n_ws, dt.device)
        call("dgrad_ln_bwd", dt, 2 * c, self._slice(Wt[2], pre + wkey), 2 * c, M, c, 2 * c, x, st,
             self._slice(P, pre + norm + ".weight"), dres, out, self._slice(dflat, pre + norm + ".weight"),
             self._slice(dflat, pre + norm + ".bias"), ws, n_ws, self.dt)


class _NAFNetFn(torch.autograd.Function):
    """The whole network as one autograd node: forward and backward run the HIP executor."""

    @staticmethod
    def forward(ctx, inp, flat, net: NAFNet):
        out, tape = net.exec_forward(inp, save=True, flat=flat.detach())
        ctx.tape = tape
        ctx.net = net
        ctx.flat = flat.detach()
        ctx.need_dx = ctx.needs_input_grad[0]
        return out

    @staticmethod
    def backward(ctx, dout):
        net: NAFNet = ctx.net
        dflat = torch.zeros_like(ctx.flat)
        dx = net.exec_backward(ctx.tape, dout.contiguous(), dflat, ctx.need_dx, flat=ctx.flat,
                               hook=net.grad_ready_hook)
        ctx.tape = None
        return dx, dflat, None
