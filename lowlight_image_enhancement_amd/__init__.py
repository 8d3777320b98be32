"""MI355X-native (gfx950) NewBP-NAFNet hot path: NAFNet fwd/bwd (Scenario B), the crosstalk-PSF physics branch
and the HybridLoss terms as hand-written HIP kernels behind a C-ABI (include/nbp.h), exposed through the
reference's Python API (RUA1027/Lowlight_Image_Enhancement: NewBP_model.*, metrics.phys_consistency).

    from lowlight_image_enhancement_amd.NewBP_model.newbp_net_arch import create_newbp_net, create_crosstalk_psf
    from lowlight_image_enhancement_amd.NewBP_model.losses import HybridLossPlus
    from lowlight_image_enhancement_amd.metrics.phys_consistency import phys_cons_srgb

`install_aliases()` registers the reference's module names (NewBP_model.*, metrics.{phys_consistency, linear, psnr,
ssim, color_error, lpips_metric}, basicsr.metrics.lowlight_metrics)
so unmodified train/eval scripts import this implementation.
"""
import sys

__version__ = "0.1.0"


def install_aliases():
    from . import NewBP_model, metrics
    from .NewBP_model import losses, newbp_layer, newbp_net_arch
    from .metrics import color_error, linear, lowlight_metrics, lpips_metric, phys_consistency, psnr, ssim
    sys.modules.setdefault("NewBP_model", NewBP_model)
    sys.modules.setdefault("NewBP_model.newbp_layer", newbp_layer)
    sys.modules.setdefault("NewBP_model.newbp_net_arch", newbp_net_arch)
    sys.modules.setdefault("NewBP_model.losses", losses)
    sys.modules.setdefault("metrics", metrics)
    sys.modules.setdefault("metrics.phys_consistency", phys_consistency)
    sys.modules.setdefault("metrics.linear", linear)
    sys.modules.setdefault("metrics.psnr", psnr)
    sys.modules.setdefault("metrics.ssim", ssim)
    sys.modules.setdefault("metrics.color_error", color_error)
    sys.modules.setdefault("metrics.lpips_metric", lpips_metric)
    sys.modules.setdefault("basicsr.metrics.lowlight_metrics", lowlight_metrics)
    from .data import data_sampler, file_client, prefetch_dataloader, sony_sid_lmdb_dataset
    sys.modules.setdefault("basicsr.data.sony_sid_lmdb_dataset", sony_sid_lmdb_dataset)
    sys.modules.setdefault("basicsr.data.prefetch_dataloader", prefetch_dataloader)
    sys.modules.setdefault("basicsr.data.data_sampler", data_sampler)
    sys.modules.setdefault("basicsr.utils.file_client", file_client)
