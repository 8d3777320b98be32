"""NewBP_model.newbp_net_arch on MI355X (reference: NewBP_model/newbp_net_arch.py:31-99)."""
from __future__ import annotations

import logging
from typing import Any, Dict, Optional, Sequence

from ..nafnet import NAFNet
from .newbp_layer import CrosstalkPSF, build_psf_kernels

logger = logging.getLogger(__name__)


def create_newbp_net(in_channels: int = 3, kernel_type: str = "panchromatic", kernel_spec: str = "P2",
                     width: Optional[int] = None, enc_blk_nums: Optional[Sequence[int]] = None,
                     middle_blk_num: Optional[int] = None, dec_blk_nums: Optional[Sequence[int]] = None,
                     nafnet_params: Optional[Dict[str, Any]] = None, **nafnet_kwargs: Any):
    """Scenario B: a plain NAFNet (no input-side K).  nafnet_params + kwargs are merged, img_channel is forced to
    in_channels (:54), kernel_type / kernel_spec are only logged (:63-73)."""
    if nafnet_params is not None and not isinstance(nafnet_params, dict):
        raise TypeError("nafnet_params must be a dictionary if provided.")
    cfg: Dict[str, Any] = {}
    if nafnet_params:
        cfg.update(nafnet_params)
    if nafnet_kwargs:
        cfg.update(nafnet_kwargs)
    cfg["img_channel"] = in_channels
    if width is not None:
        cfg["width"] = width
    if enc_blk_nums is not None:
        cfg["enc_blk_nums"] = list(enc_blk_nums)
    if middle_blk_num is not None:
        cfg["middle_blk_num"] = middle_blk_num
    if dec_blk_nums is not None:
        cfg["dec_blk_nums"] = list(dec_blk_nums)
    net = NAFNet(**cfg)
    logger.info("[NewBP-Net] Created (Scenario B: no input-side K). kernel_type='%s', kernel_spec='%s', in_channels=%s, "
                "width=%s, enc_blks=%s, middle=%s, dec_blks=%s.", kernel_type, kernel_spec, in_channels,
                cfg.get("width"), cfg.get("enc_blk_nums"), cfg.get("middle_blk_num"), cfg.get("dec_blk_nums"))
    return net


def create_crosstalk_psf(psf_mode: str = "mono", kernel_spec: str = "P2"):
    """newbp_net_arch.py:88-99."""
    if psf_mode not in {"mono", "rgb"}:
        raise ValueError("psf_mode must be 'mono' or 'rgb'")
    return CrosstalkPSF(mode=psf_mode, kernels=build_psf_kernels(psf_mode, kernel_spec))


def NewBPNAFNet(**kwargs: Any):
    """BasicSR registry alias (NAFNet_base/basicsr/models/archs/newbp_nafnet_arch.py:47-51)."""
    return create_newbp_net(**kwargs)
