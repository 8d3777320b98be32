"""Oracle: crosstalk PSF, exposure alignment, physics-consistency losses and metrics.

Test infrastructure only (see oracle/__init__.py).
"""
from __future__ import annotations

import warnings

import torch
import torch.nn.functional as F

# NewBP_model/newbp_layer.py:140-164 — corner / edge / centre weights of the fixed 3x3 tables.
_TABLES = {
    "P2": (0.0100, 0.0200, 0.8800),
    "R": (0.0117, 0.0233, 0.8600),
    "G": (0.0100, 0.0200, 0.8800),
    "B": (0.0083, 0.0167, 0.9000),
}


def _table(name):
    c, e, m = _TABLES[name]
    return torch.tensor([[c, e, c], [e, m, e], [c, e, c]], dtype=torch.float32).view(1, 1, 3, 3)


# "Stressed" RGB crosstalk family (R > G > B leakage) — a BUILD artefact, not a reference table: the reference only
# describes it (README.md:24,64,214).  S1/S2/S3 leak 1.5x/2x/2.5x of B2's off-centre mass (R .14, G .12,
# B .10) with B2's edge:corner = 2:1 split: corner = leak / 12, edge = leak / 6, centre = 1 - leak.
STRESSED = {f"S{i}": tuple(round(f * l, 6) for l in (0.14, 0.12, 0.10)) for i, f in ((1, 1.5), (2, 2.0), (3, 2.5))}


def _stressed(spec: str, leak: float) -> torch.Tensor:
    c, e, m = leak / 12.0, leak / 6.0, 1.0 - leak
    return torch.tensor([[c, e, c], [e, m, e], [c, e, c]], dtype=torch.float32).view(1, 1, 3, 3)


def build_psf_kernels(mode: str, kernel_spec: str = "P2") -> torch.Tensor:
    """newbp_layer.py:129-173: mono/P2 -> [1,1,3,3]; rgb/B2 -> [3,1,3,3]; ValueError otherwise."""
    if mode not in ("mono", "rgb"):
        raise ValueError("mode must be 'mono' or 'rgb'")
    if mode == "mono":
        if kernel_spec != "P2":
            raise ValueError("mono mode expects kernel_spec 'P2'")
        return _table("P2")
    if kernel_spec in STRESSED:
        return torch.cat([_stressed(kernel_spec, leak) for leak in STRESSED[kernel_spec]], 0)
    if kernel_spec != "B2":
        raise ValueError("rgb mode expects kernel_spec 'B2' (or the stressed family 'S1', 'S2', 'S3')")
    return torch.cat([_table("R"), _table("G"), _table("B")], 0)


def normalize_psf(k: torch.Tensor) -> torch.Tensor:
    """CrosstalkPSF.__init__ (newbp_layer.py:102-106): per-kernel k / clamp_min(sum, 1e-12)."""
    s = k.reshape(k.shape[0], -1).sum(dim=1, keepdim=True).clamp_min(1e-12)
    return k / s.view(-1, 1, 1, 1)


def psf_apply(x: torch.Tensor, k: torch.Tensor) -> torch.Tensor:
    """CrosstalkPSF.forward (newbp_layer.py:109-126): depthwise groups=3, zero pad 1."""
    assert x.shape[1] == 3
    if k.shape[0] == 1:
        k = k.expand(3, 1, 3, 3)
    return F.conv2d(x, k, bias=None, stride=1, padding=1, groups=3)


def align_exposure_srgb(a: torch.Tensor, ratio) -> torch.Tensor:
    """losses.py:195-203: float -> tensor, 0-d -> [1], 1-d -> [B,1,1,1]; clamp(a*ratio, 0, 1)."""
    if not torch.is_tensor(ratio):
        ratio = torch.tensor(ratio, dtype=a.dtype, device=a.device)
    if ratio.dim() == 0:
        ratio = ratio.view(1)
    if ratio.dim() == 1:
        ratio = ratio.view(-1, 1, 1, 1)
    return (a * ratio).clamp(0.0, 1.0)


def phys_srgb_loss(bhat, a, ratio, k_norm) -> torch.Tensor:
    """PhysicalConsistencyLossSRGB.forward (losses.py:217-220): L1(PSF(bhat), align(a))."""
    return (psf_apply(bhat, k_norm) - align_exposure_srgb(a, ratio)).abs().mean()


def phys_raw_loss(bhat_raw, a_raw, ratio, k, clamp_align=True) -> torch.Tensor:
    """PhysicsConsistencyLoss.forward (losses.py:173-192): replicate pad, un-normalised K."""
    if ratio.dim() == 1:
        ratio = ratio.view(-1, 1, 1, 1)
    a_al = a_raw * ratio
    if clamp_align:
        a_al = a_al.clamp(0.0, 1.0)
    kh, kw = k.shape[-2:]
    x = F.pad(bhat_raw, (kw // 2, kw // 2, kh // 2, kh // 2), mode="replicate")
    C = bhat_raw.shape[1]
    if k.shape[0] == 1 and C > 1:
        k = k.expand(C, 1, kh, kw)
    groups = C if k.shape[0] == C else 1
    if groups == 1 and k.shape[1] == 1 and C != 1:
        k = k.expand(k.shape[0], C, kh, kw)
    return (F.conv2d(x, k, groups=groups) - a_al).abs().mean()


# ---- metrics/phys_consistency.py restated (no-grad metric form) ---------------------------------
def _prepare_psf(psf, cin, cout, normalize, nonneg, eps):
    """phys_consistency.py:75-127."""
    if psf.ndim == 2:
        psf = psf[None, None]
    if psf.ndim != 4:
        raise ValueError("psf must be [C_out, C_in, kh, kw]")
    co, ci, kh, kw = psf.shape
    if co != cout or ci != cin or kh < 1 or kw < 1 or kh % 2 == 0 or kw % 2 == 0:
        raise ValueError("bad psf shape")
    psf = psf.float()
    if nonneg:
        psf = psf.clamp_min(0)
    if normalize:
        s = psf.reshape(co, -1).sum(dim=1)
        z = s.abs() < eps
        if z.any():
            warnings.warn("PSF channel sums near zero", RuntimeWarning)
        psf = psf / torch.where(z, torch.ones_like(s), s).view(co, 1, 1, 1)
    return psf


def _expand_ratio(r, ref):
    """phys_consistency.py:160-190."""
    r = r.to(ref.dtype) if torch.is_tensor(r) else torch.tensor(float(r), dtype=ref.dtype)
    n = ref.shape[0]
    if r.ndim == 0:
        return r.view(1, 1, 1, 1).expand(n, 1, 1, 1)
    if r.ndim == 1:
        if r.shape[0] != n:
            raise ValueError("ratio length")
        return r.view(n, 1, 1, 1)
    if r.ndim == 4:
        if r.shape[0] != n:
            raise ValueError("ratio batch")
        if r.shape[1] == 1 and ref.shape[1] > 1:
            return r.expand(n, ref.shape[1], r.shape[2], r.shape[3])
        if r.shape[1] not in (1, ref.shape[1]):
            raise ValueError("ratio channels")
        return r
    raise ValueError("ratio rank")


def phys_cons(pred, obs, psf, ratio, *, clamp01, reduction="mean", padding="reflect", normalize_psf=True,
              enforce_nonnegative=False, crop="valid", robust="none", return_map=False, eps=1e-12):
    """_phys_cons_core (phys_consistency.py:193-255) for phys_cons_raw (:260) and phys_cons_srgb (:323)."""
    if pred.ndim == 3:
        pred, obs = pred[None], obs[None]
    pred, obs = pred.float(), obs.float()
    k = _prepare_psf(psf, pred.shape[1], obs.shape[1], normalize_psf, enforce_nonnegative, eps)
    kh, kw = k.shape[-2:]
    pad = (kw // 2, kw // 2, kh // 2, kh // 2)
    if padding == "zeros":
        y = F.conv2d(pred, k, padding=(kh // 2, kw // 2))
    else:
        y = F.conv2d(F.pad(pred, pad, mode=padding), k)
    r = _expand_ratio(ratio, y)
    if r.shape[1] == 1 and y.shape[1] != 1:
        r = r.expand(y.shape[0], y.shape[1], r.shape[2], r.shape[3])
    y = y * r
    if clamp01:
        y = y.clamp(0.0, 1.0)
    o = obs
    if crop == "valid":
        ph, pw = kh // 2, kw // 2
        if ph > 0:
            y, o = y[..., ph:-ph, :], o[..., ph:-ph, :]
        if pw > 0:
            y, o = y[..., :, pw:-pw], o[..., :, pw:-pw]
    d = y - o
    lm = torch.sqrt(d * d + eps * eps) if robust == "charbonnier" else d.abs()
    per = lm.flatten(1).mean(dim=1)
    m = {"none": per, "mean": per.mean(0) if reduction == "mean" else None}.get(reduction)
    if reduction == "sum":
        m = per.sum(0)
    return (m, d.abs()) if return_map else m
