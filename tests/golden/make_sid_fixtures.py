"""Copy the reference's own SID debug fixtures (data files, not code) into tests/golden/sid/.

Source: <reference>/data/debug_sid/ — manifest_sid_debug.json, short/*.png, long/*.png and the
train_small_{short,long}.lmdb environments (data.mdb + meta_info.txt).  Run once in the container that holds the
reference; the GPU box and the tests only read the copies.
"""
import os
import shutil
import sys

SRC = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/data/debug_sid"
DST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sid")

FILES = ["manifest_sid_debug.json", "short/debugpair1_00_0.1s.png", "short/debugpair2_00_0.1s.png",
         "long/debugpair1_00_1s.png", "long/debugpair2_00_1s.png",
         "train_small_short.lmdb/data.mdb", "train_small_short.lmdb/meta_info.txt",
         "train_small_long.lmdb/data.mdb", "train_small_long.lmdb/meta_info.txt"]

for f in FILES:
    os.makedirs(os.path.dirname(os.path.join(DST, f)), exist_ok=True)
    shutil.copyfile(os.path.join(SRC, f), os.path.join(DST, f))
    os.chmod(os.path.join(DST, f), 0o644)
print("copied", len(FILES), "files to", DST)
