"""VGPR / AGPR / SGPR / LDS / spill use of the gfx950 kernels in a built object (in-tree obj/ of build.py):
python scripts/kernel_resources.py gemm_bf16 [name-substring ...]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
obj = os.path.join(os.path.dirname(__file__), "..", "lowlight_image_enhancement_amd", "_lib", "obj", sys.argv[1] + ".o")
pats = sys.argv[2:]
with tempfile.TemporaryDirectory() as d:
    fb, co = os.path.join(d, "fb.bin"), os.path.join(d, "g.co")
    subprocess.check_call([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj,
                           os.path.join(d, "copy.o")])  # (without an output file objcopy rewrites its input)
    subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                           "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
    notes = subprocess.check_output([f"{LLVM}/llvm-readelf", "--notes", co], text=True)
for blk in re.split(r"\n\s+- \.agpr_count", notes)[1:]:
    blk = ".agpr_count" + blk
    f = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, "?"])[1]  # noqa: E731
    name = f("name")
    if pats and not any(p in name for p in pats):
        continue
    print(f"{name[:96]:96s} vgpr {f('vgpr_count'):>4s} agpr {f('agpr_count'):>3s} sgpr {f('sgpr_count'):>3s} "
          f"lds {f('group_segment_fixed_size'):>6s} spill {f('vgpr_spill_count')} priv {f('private_segment_fixed_size')}")
