"""Build an A/B variant of the library with extra preprocessor flags into lowlight_image_enhancement_amd/_lib/<name>/,
selected at run time with NBP_LIB (never the production library).
    python scripts/build_variant.py NAME -DFLAG=VALUE [...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lowlight_image_enhancement_amd import build as B  # noqa: E402

name, flags = sys.argv[1], sys.argv[2:]
assert name and all(f.startswith("-D") for f in flags), "usage: build_variant.py NAME -DFLAG=VALUE ..."
B.OUT_DIR = os.path.join(B.PKG, "_lib", name)
B.LIB = os.path.join(B.OUT_DIR, "liblowlight_nbp.so")
B.CFLAGS = B.CFLAGS + flags
print(B.build_library())
