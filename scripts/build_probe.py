"""Build the timeline-probe variant of the library (-DNBP_GEMM_PROBE: gemm_glds_kernel stamps, gemm16_impl.h) into
lowlight_image_enhancement_amd/_lib/probe/liblowlight_nbp.so, selected at run time with NBP_LIB (scripts/gemm_timeline.py).
Never the production library.
    python scripts/build_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lowlight_image_enhancement_amd import build as B  # noqa: E402

MINBLK = os.environ.get("MINBLK")  # the tile-choice threshold (blocks per launch) of this build, default 512
NS5 = os.environ.get("NS5") == "1"  # 5-deep LDS-DMA rings where they fit
B.OUT_DIR = os.path.join(B.PKG, "_lib", "probe" + (MINBLK or "") + ("ns5" if NS5 else ""))
B.LIB = os.path.join(B.OUT_DIR, "liblowlight_nbp.so")
B.CFLAGS = B.CFLAGS + ["-DNBP_GEMM_PROBE=1"] + ([f"-DNBP_GEMM_MINBLK={MINBLK}"] if MINBLK else []) + (
    ["-DNBP_GEMM_NS5=1"] if NS5 else [])
print(B.build_library())
