"""SID input path (reference NAFNet_base/basicsr/data/sony_sid_lmdb_dataset.py,
basicsr/utils/file_client.py, basicsr/data/prefetch_dataloader.py).

Pins: the reference's own fixtures (tests/golden/sid, copied from data/debug_sid by tests/golden/make_sid_fixtures.py)
— PNGs decoded by PIL, LMDB values that decode to the same pixels as the files on disk, the manifest.  Beyond them,
the native decoder / reader are checked against the oracle restatement (oracle/sid_input.py) on synthetic PNGs
(every filter, Adam7, 16-bit, palettes) and LMDB environments with branch levels, written by tests/sid_fixtures.py.
The device conversion is bitwise against the oracle's numpy float32 arithmetic.
"""
import io
import json
import os

import numpy as np
import pytest
import torch

from oracle import sid_input as osid
from sid_fixtures import encode_png, write_lmdb

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "sid")
PNGS = ["short/debugpair1_00_0.1s.png", "short/debugpair2_00_0.1s.png", "long/debugpair1_00_1s.png",
        "long/debugpair2_00_1s.png"]


def _read(rel):
    with open(os.path.join(GOLD, rel), "rb") as f:
        return f.read()


# ------------------------------------------------------------------------------------------- oracle pinning (CPU)
def test_oracle_png_matches_pil_on_reference_fixtures():
    from PIL import Image
    for rel in PNGS:
        ref = np.array(Image.open(os.path.join(GOLD, rel))).astype(np.uint16) * 257
        assert np.array_equal(osid.png_decode(_read(rel)), ref), rel


def test_oracle_lmdb_values_decode_to_the_disk_pngs():
    for kind, key, disk in (("short", "debugpair1_00_0.1s.png", "short/debugpair1_00_0.1s.png"),
                            ("long", "debugpair1_00_1s.png", "long/debugpair1_00_1s.png")):
        db = osid.LmdbReader(os.path.join(GOLD, f"train_small_{kind}.lmdb"))
        meta = open(os.path.join(GOLD, f"train_small_{kind}.lmdb", "meta_info.txt")).read().split()[0]
        assert meta == key + ".png" and db.entries == 1
        val = db.get(key.encode())
        assert val[:8] == b"\x89PNG\r\n\x1a\n"
        assert np.array_equal(osid.png_decode(val), osid.png_decode(_read(disk)))
        assert db.get(b"debugpair9_00_1s.png") is None and db.get(b"") is None


@pytest.mark.parametrize("kind", ["rgb8", "pal4", "pal8", "rgb8_interlaced"])
def test_oracle_png_matches_pil_on_synthetic(kind):
    from PIL import Image
    rng = np.random.default_rng(len(kind))
    H, W = 19, 23
    if kind.startswith("rgb8"):
        s = rng.integers(0, 256, (H, W, 3))
        png = encode_png(s, 8, 2, interlace=kind.endswith("interlaced"), rng=rng)
    else:
        depth = int(kind[3:])
        pal = rng.integers(0, 256, (1 << depth, 3))
        s = rng.integers(0, 1 << depth, (H, W, 1))
        png = encode_png(s, depth, 3, palette=pal, rng=rng)
    ref = np.array(Image.open(io.BytesIO(png)).convert("RGB")).astype(np.uint16) * 257
    assert np.array_equal(osid.png_decode(png), ref)


def test_oracle_png16_high_bytes_match_pil():
    """PIL reads 16-bit RGB as 8-bit (the high byte): pins the 16-bit sample order of the oracle."""
    from PIL import Image
    rng = np.random.default_rng(3)
    s = rng.integers(0, 65536, (11, 13, 3))
    png = encode_png(s, 16, 2, rng=rng)
    dec = osid.png_decode(png)
    assert np.array_equal(dec, s.astype(np.uint16))
    assert np.array_equal(dec >> 8, np.array(Image.open(io.BytesIO(png))).astype(np.uint16))


# --------------------------------------------------------------------------------------- native host code (CPU)
def _synthetic_pngs():
    rng = np.random.default_rng(11)
    cases = []
    for H, W in ((1, 1), (3, 7), (37, 29), (64, 5)):
        for depth in (8, 16):
            for inter in (False, True):
                s = rng.integers(0, 1 << depth, (H, W, 3))
                cases.append((f"rgb{depth}_{H}x{W}_i{int(inter)}", encode_png(s, depth, 2, interlace=inter, rng=rng,
                                                                             idat_split=97)))
        for depth in (1, 2, 4, 8):
            pal = rng.integers(0, 256, (1 << depth, 3))
            s = rng.integers(0, 1 << depth, (H, W, 1))
            cases.append((f"pal{depth}_{H}x{W}", encode_png(s, depth, 3, palette=pal, rng=rng,
                                                            interlace=bool(depth & 2))))
    for ft in range(5):
        s = rng.integers(0, 65536, (9, 17, 3))
        cases.append((f"filter{ft}", encode_png(s, 16, 2, filters=ft)))
    return cases


def test_native_png_decoder_matches_oracle():
    from lowlight_image_enhancement_amd.data.sony_sid_lmdb_dataset import _load_png_uint16, png_shape
    rng = np.random.default_rng(5)
    for name, png in _synthetic_pngs() + [(rel, _read(rel)) for rel in PNGS]:
        ref = osid.png_decode(png)
        assert png_shape(png) == ref.shape, name
        assert np.array_equal(_load_png_uint16(png), ref), name
        H, W, _ = ref.shape
        for _ in range(3):  # crop windows decoded directly
            ch, cw = int(rng.integers(1, H + 1)), int(rng.integers(1, W + 1))
            top, left = int(rng.integers(0, H - ch + 1)), int(rng.integers(0, W - cw + 1))
            got = _load_png_uint16(png, (top, left, ch, cw))
            assert np.array_equal(got, ref[top:top + ch, left:left + cw]), (name, top, left, ch, cw)


def test_native_png_rejects_what_the_reference_rejects():
    from lowlight_image_enhancement_amd.data.sony_sid_lmdb_dataset import _load_png_uint16
    rng = np.random.default_rng(2)
    good = encode_png(rng.integers(0, 256, (8, 8, 3)), 8, 2)
    with pytest.raises(ValueError, match="empty buffer"):
        _load_png_uint16(None)
    idat = good.index(b"IDAT") + 10
    for bad in (b"not a png", good[:-20], good[:idat] + bytes([good[idat] ^ 1]) + good[idat + 1:],
                good[:20] + bytes([good[20] ^ 1]) + good[21:]):  # truncated, IDAT and IHDR CRC errors
        with pytest.raises(ValueError):
            _load_png_uint16(bad)
    # a CRC error in an ancillary chunk (tEXt) is discarded, as libpng does by default
    text = good.index(b"tEXt") + 6
    assert np.array_equal(_load_png_uint16(good[:text] + bytes([good[text] ^ 1]) + good[text + 1:]),
                          _load_png_uint16(good))
    # cv2 IMREAD_UNCHANGED shapes the reference rejects with ValueError (:52-55): gray, gray+alpha, RGBA, palette+tRNS
    rejected = [(encode_png(rng.integers(0, 65536, (4, 5, 1)), 16, 0), (4, 5, 1)),
                (encode_png(rng.integers(0, 256, (4, 5, 2)), 8, 4), (4, 5, 4)),
                (encode_png(rng.integers(0, 256, (4, 5, 4)), 8, 6), (4, 5, 4)),
                (encode_png(rng.integers(0, 4, (4, 5, 1)), 2, 3, palette=rng.integers(0, 256, (4, 3)), trns=True),
                 (4, 5, 4))]
    for png, shape in rejected:
        with pytest.raises(ValueError, match=r"Expected 3-channel image, got shape \(4, 5, [14]\)"):
            _load_png_uint16(png)


def test_native_decode_batch_threads():
    from lowlight_image_enhancement_amd.data.sony_sid_lmdb_dataset import _load_png_uint16, decode_batch
    rng = np.random.default_rng(9)
    pngs = [encode_png(rng.integers(0, 65536, (40, 50, 3)), 16, 2, rng=rng, interlace=bool(i % 3 == 0))
            for i in range(12)]
    wins = [(int(rng.integers(0, 9)), int(rng.integers(0, 19)), 32, 32) for _ in pngs]
    one = decode_batch(pngs, wins, nthreads=1)
    many = decode_batch(pngs, wins, nthreads=8)
    assert np.array_equal(one, many)
    for i, (p, w) in enumerate(zip(pngs, wins)):
        assert np.array_equal(one[i], _load_png_uint16(p, w))
    with pytest.raises(ValueError):
        decode_batch(pngs[:2], [wins[0], (0, 0, 16, 16)])


def test_native_lmdb_reader_on_reference_fixtures():
    from lowlight_image_enhancement_amd.data import FileClient
    fc = FileClient("lmdb", db_paths=[os.path.join(GOLD, "train_small_short.lmdb"),
                                      os.path.join(GOLD, "train_small_long.lmdb", "data.mdb")],
                    client_keys=["short", "long"])
    for ck, key in (("short", "debugpair1_00_0.1s.png"), ("long", "debugpair1_00_1s.png")):
        ref = osid.LmdbReader(os.path.join(GOLD, f"train_small_{ck}.lmdb")).get(key.encode())
        assert fc.get(key, ck) == ref
        assert fc.client.entries(ck) == 1
    assert fc.get("debugpair2_00_0.1s.png", "short") is None
    with pytest.raises(AssertionError):
        fc.get("x", "nope")
    with pytest.raises(ValueError):
        FileClient("memcached2")


@pytest.mark.parametrize("n,fanout", [(1, None), (40, None), (700, None), (700, 3)])
def test_native_lmdb_reader_multilevel_trees(tmp_path, n, fanout):
    """Leaves, branch levels (fanout 3 gives a deep tree), inline and overflow values, absent keys between,
    before and after the stored ones."""
    from lowlight_image_enhancement_amd.data.file_client import LmdbBackend
    rng = np.random.default_rng(n)
    items = {}
    for i in range(n):
        k = f"img_{int(rng.integers(0, 10 ** 6)):07d}_{i}.png".encode()
        size = int(rng.choice([0, 5, 300, 601, 5000, 9000]))
        items[k] = rng.integers(0, 256, size).astype(np.uint8).tobytes()
    path = str(tmp_path / "data.mdb")
    write_lmdb(path, items, fanout=fanout)
    be = LmdbBackend(str(tmp_path), client_keys="db")
    ref = osid.LmdbReader(str(tmp_path))
    assert be.entries("db") == n
    for k, v in items.items():
        assert be.get(k.decode(), "db") == v == ref.get(k)
    for probe in (b"", b"a", b"img_", b"img_9999999", b"zzz", sorted(items)[0] + b"x", sorted(items)[-1] + b"\x00"):
        if probe not in items:
            assert be.get(probe.decode(), "db") is None and ref.get(probe) is None
    be.close()


def test_native_lmdb_rejects_corrupt_files(tmp_path):
    from lowlight_image_enhancement_amd._lib import NBPError
    from lowlight_image_enhancement_amd.data.file_client import LmdbBackend
    (tmp_path / "small").write_bytes(b"\x00" * 100)
    (tmp_path / "zeros").write_bytes(b"\x00" * 3 * 4096)
    for name in ("small", "zeros", "missing"):
        with pytest.raises(NBPError):
            LmdbBackend(str(tmp_path / name))


# ------------------------------------------------------------------------------------------------ dataset (CPU)
def _opt(tmp_path, **kw):
    opt = {"manifest_path": os.path.join(GOLD, "manifest_sid_debug.json"), "phase": "train", "subset": "train_small",
           "io_backend": {"type": "lmdb", "db_paths": [os.path.join(GOLD, "train_small_short.lmdb"),
                                                        os.path.join(GOLD, "train_small_long.lmdb")],
                          "client_keys": ["short", "long"]},
           "patch_size": 24, "samples_per_pair": 5, "seed": 123}
    opt.update(kw)
    return opt


def test_dataset_options_and_errors(tmp_path):
    from lowlight_image_enhancement_amd.data import SonySIDLMDBDataset
    ds = SonySIDLMDBDataset(_opt(tmp_path))
    assert len(ds) == 5 and ds.io_backend_type == "lmdb"
    with pytest.raises(FileNotFoundError):
        SonySIDLMDBDataset(_opt(tmp_path, manifest_path=str(tmp_path / "none.json")))
    with pytest.raises(RuntimeError):
        SonySIDLMDBDataset(_opt(tmp_path, subset="test"))
    with pytest.raises(RuntimeError):
        SonySIDLMDBDataset(_opt(tmp_path, allowed_pair_ids=["debugpair2_00"]))
    with pytest.raises(KeyError):
        SonySIDLMDBDataset(_opt(tmp_path, io_backend={}))
    with pytest.raises(KeyError):
        SonySIDLMDBDataset(_opt(tmp_path, io_backend={"type": "lmdb", "db_paths": []}))
    with pytest.raises(ValueError):
        SonySIDLMDBDataset(_opt(tmp_path, io_backend={"type": "s3"}))
    with pytest.raises(FileNotFoundError):
        SonySIDLMDBDataset(_opt(tmp_path, io_backend={"type": "disk", "paths": {"short": str(tmp_path / "a"),
                                                                                 "long": str(tmp_path / "b")}}))
    with pytest.raises(ValueError, match="Patch size 65 exceeds"):
        SonySIDLMDBDataset(_opt(tmp_path, patch_size=65))[0]
    # legacy short_lmdb / long_lmdb keys
    legacy = _opt(tmp_path, io_backend={})
    legacy.update(short_lmdb=os.path.join(GOLD, "train_small_short.lmdb"),
                  long_lmdb=os.path.join(GOLD, "train_small_long.lmdb"))
    assert len(SonySIDLMDBDataset(legacy)) == 5


@pytest.mark.parametrize("backend,phase,random_crop", [("lmdb", "train", True), ("disk", "train", False),
                                                       ("disk", "val", True)])
def test_dataset_samples_match_reference_arithmetic(tmp_path, backend, phase, random_crop):
    """__getitem__ / get_batch: the crop draws of the reference's rng (top, then left, per sample) and the crops
    of the decoded arrays, for the LMDB and disk backends, train (random / centre crop) and val (no crop)."""
    from lowlight_image_enhancement_amd.data import SonySIDLMDBDataset
    kw = dict(phase=phase, random_crop=random_crop, return_metadata=True)
    if backend == "disk":
        kw["io_backend"] = {"type": "disk", "paths": {"short": os.path.join(GOLD, "short"),
                                                      "long": os.path.join(GOLD, "long")}}
    if phase == "val":
        kw.update(subset="val_small", samples_per_pair=1)
    ds = SonySIDLMDBDataset(_opt(tmp_path, **kw))
    manifest = json.load(open(os.path.join(GOLD, "manifest_sid_debug.json")))
    entry = [m for m in manifest if m["subset"] == ds.subset][0]
    s_full = osid.png_decode(_read("short/" + entry["short_key"]))
    l_full = osid.png_decode(_read("long/" + entry["long_key"]))
    rng = np.random.default_rng(123)
    samples = [ds[i] for i in range(len(ds))]
    for smp in samples:
        win = osid.crop_window(rng, 64, 64, 24, phase, random_crop)
        t, l_, h, w = win
        assert np.array_equal(smp["lq_u16"].numpy().view(np.uint16), s_full[t:t + h, l_:l_ + w])
        assert np.array_equal(smp["gt_u16"].numpy().view(np.uint16), l_full[t:t + h, l_:l_ + w])
        assert smp["expo_ratio"].shape == (1, 1, 1) and float(smp["expo_ratio"]) == entry["exposure_ratio"]
        assert smp["pair_id"] == entry["pair_id"] == smp["key"] and smp["lq_path"] == entry["short_key"]
        assert smp["metadata"]["exposure_ratio"] == entry["exposure_ratio"]
    # get_batch == default_collate(__getitem__) on a fresh dataset with the same seed
    ds2 = SonySIDLMDBDataset(_opt(tmp_path, **kw))
    batch = ds2.get_batch(list(range(len(ds2))), nthreads=4)
    assert torch.equal(batch["lq_u16"], torch.stack([s["lq_u16"] for s in samples]))
    assert torch.equal(batch["gt_u16"], torch.stack([s["gt_u16"] for s in samples]))
    assert batch["expo_ratio"].shape == (len(ds2), 1, 1, 1) and batch["pair_id"] == [s["pair_id"] for s in samples]


# -------------------------------------------------------------------------------------------------- device (GPU)
@pytest.mark.gpu
@pytest.mark.parametrize("B,H,W", [(3, 17, 300), (16, 64, 64), (1, 1, 1)])
def test_sid_to_float_bitwise_vs_oracle(B, H, W):
    from lowlight_image_enhancement_amd._lib import call
    rng = np.random.default_rng(B * H + W)
    s = rng.integers(0, 65536, (B, H, W, 3)).astype(np.uint16)
    l_ = rng.integers(0, 65536, (B, H, W, 3)).astype(np.uint16)
    s[0, 0, 0] = [0, 65535, 6553]
    ratios = [1.0, 10.0, 100.0, 250.0, 300.0, 0.5, 3.3, 1e-3][:B] + [7.0] * max(0, B - 8)
    dev = torch.device("cuda")
    s16 = torch.from_numpy(s.view(np.int16)).to(dev)
    l16 = torch.from_numpy(l_.view(np.int16)).to(dev)
    r = torch.tensor(ratios, dtype=torch.float32, device=dev)
    lq, sraw, lraw = (torch.empty(B, 3, H, W, device=dev) for _ in range(3))
    call("sid_to_float", s16, l16, r, B, H, W, lq, sraw, lraw)
    for b in range(B):
        ref = osid.getitem_arrays(s[b], l_[b], ratios[b], (0, 0, H, W))
        assert np.array_equal(lq[b].cpu().numpy(), ref["lq"]), b
        assert np.array_equal(sraw[b].cpu().numpy(), ref["short_raw"])
        assert np.array_equal(lraw[b].cpu().numpy(), ref["long_raw"])


@pytest.mark.gpu
def test_prefetcher_delivers_the_reference_batch(tmp_path):
    """Dataset -> DataLoader(pin_memory) -> CUDAPrefetcher: every batch dict equals the reference's __getitem__
    arithmetic (oracle) on the same crops, bit for bit, with the reference's keys and aliases."""
    from lowlight_image_enhancement_amd.data import CUDAPrefetcher, SonySIDLMDBDataset
    ds = SonySIDLMDBDataset(_opt(tmp_path, samples_per_pair=6))
    loader = torch.utils.data.DataLoader(ds, batch_size=2, shuffle=False, num_workers=0, pin_memory=True)
    pf = CUDAPrefetcher(loader, {"num_gpu": 1})
    s_full = osid.png_decode(_read("short/debugpair1_00_0.1s.png"))
    l_full = osid.png_decode(_read("long/debugpair1_00_1s.png"))
    rng = np.random.default_rng(123)
    n = 0
    while True:
        batch = pf.next()
        if batch is None:
            break
        for k in ("lq", "gt", "short", "long", "short_raw", "long_raw", "short_obs", "expo_ratio", "pair_id",
                  "lq_path", "gt_path", "key"):
            assert k in batch, k
        assert batch["short"] is batch["lq"] and batch["short_obs"] is batch["lq"] and batch["long"] is batch["gt"]
        assert batch["lq"].shape == (2, 3, 24, 24) and batch["expo_ratio"].shape == (2, 1, 1, 1)
        for b in range(2):
            win = osid.crop_window(rng, 64, 64, 24, "train", True)
            ref = osid.getitem_arrays(s_full, l_full, 10.0, win)
            for k in ("lq", "gt", "short_raw", "long_raw"):
                assert np.array_equal(batch[k][b].cpu().numpy(), ref[k]), k
        n += 1
    assert n == 3


def test_enlarged_sampler_shards_and_loader(tmp_path):
    """EnlargedSampler (basicsr/data/data_sampler.py): per-rank strided shards of one epoch-seeded permutation,
    disjoint across ranks and covering the enlarged epoch; create_dataloader's train / val contracts."""
    from lowlight_image_enhancement_amd.data import EnlargedSampler, SonySIDLMDBDataset, create_dataloader
    ds = SonySIDLMDBDataset(_opt(tmp_path, samples_per_pair=7))
    for world, ratio in ((1, 1), (2, 3), (4, 100)):
        shards = [list(EnlargedSampler(ds, world, r, ratio)) for r in range(world)]
        total = -(-len(ds) * ratio // world) * world
        perm = torch.randperm(total, generator=torch.Generator().manual_seed(0)).tolist()
        for r, sh in enumerate(shards):
            assert len(sh) == total // world and sh == [v % len(ds) for v in perm][r::world]
    s = EnlargedSampler(ds, 2, 1, 3)
    s.set_epoch(5)
    assert list(s) != list(EnlargedSampler(ds, 2, 1, 3))
    dl = create_dataloader(ds, {"phase": "train", "batch_size_per_gpu": 2, "num_worker_per_gpu": 0}, num_gpu=1,
                           dist=True, sampler=EnlargedSampler(ds, 2, 0, 1), seed=0)
    batches = list(dl)
    assert len(batches) == 2 and batches[0]["lq_u16"].shape == (2, 24, 24, 3)  # drop_last: 4 of 4 samples
    val = create_dataloader(ds, {"phase": "val"})
    assert val.batch_size == 1
    with pytest.raises(ValueError):
        create_dataloader(ds, {"phase": "other"})
    with pytest.raises(ValueError):
        create_dataloader(ds, {"phase": "val", "prefetch_mode": "cpu"})
