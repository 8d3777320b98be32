"""A/B of the executor's fusion attributes in the bench step: runs bench.py with NAFNet attributes overridden after
construction, e.g.  python scripts/ab_attr.py fuse_c1dw=0 fuse_ffn=1 -- --quick --steps 20 --warmup 5
(the attributes are the ones nafnet.py documents: fuse_c1dw, fuse_ffn, fuse_ln_fwd, group_wgrad, sg_rc, sg_rc_wg)."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
args = sys.argv[1:]
cut = args.index("--") if "--" in args else len(args)
over = dict(a.split("=", 1) for a in args[:cut])
from lowlight_image_enhancement_amd import nafnet  # noqa: E402

_init = nafnet.NAFNet.__init__


def _patched(self, *a, **k):
    _init(self, *a, **k)
    for key, v in over.items():
        if not hasattr(self, key):
            raise SystemExit(f"unknown attribute {key}")
        setattr(self, key, v not in ("0", "false", "False"))


nafnet.NAFNet.__init__ = _patched
sys.argv = [os.path.join(ROOT, "bench.py")] + args[cut + 1:]
runpy.run_path(sys.argv[0], run_name="__main__")
