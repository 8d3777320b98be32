"""Narrow 16-bit weight gradients on the full-width kernel (wgrad_narrow_full, csrc/gemm.hip) through the C-ABI
nbp_wgrad_f32: every shape the level-0 / 1 NAFBlocks and down / up convs issue, plus ragged row counts, against a
float64 reference of dW = G^T X (with the per-image column scale of the SCA operand, NAFNet_arch.py:67) and
db = colsum G.  The reference computes these gradients with torch autograd over the same operands (NAFNet_arch.py:
59-80, 117-122, 148-149)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _check(dW, db, ref, bref, M):
    tol = 2e-6 * max(1.0, (M / 4096) ** 0.5)
    err = (dW.double() - ref.reshape(-1)).abs().max().item() / (ref.abs().max().item() + 1e-12)
    berr = (db.double() - bref).abs().max().item() / (bref.abs().max().item() + 1e-12)
    assert err <= tol and berr <= tol, (err, berr)


@pytest.mark.parametrize("M,N,K,rows,dtype", [
    (16384, 128, 64, 0, 1), (16384 + 61, 128, 64, 0, 2), (8192, 64, 64, 0, 1), (3 * 64 + 5, 64, 32, 0, 1),
    (8192, 32, 64, 0, 2), (4096, 128, 32, 0, 1), (32, 32, 32, 0, 1),
    (4 * 4096, 32, 32, 4096, 1), (3 * 1024, 64, 64, 1024, 2), (2 * 64, 64, 32, 64, 1)])
def test_wgrad_full_plain_and_scaled(dev, M, N, K, rows, dtype):
    from lowlight_image_enhancement_amd._lib import call, query
    ht = torch.bfloat16 if dtype == 1 else torch.float16
    gen = torch.Generator(device=dev).manual_seed(M * 7 + N + K + dtype)
    G = torch.randn(M, N, device=dev, generator=gen).to(ht)
    X = torch.randn(M, K, device=dev, generator=gen).to(ht)
    nimg = (M + rows - 1) // rows if rows else 1
    sc = torch.rand(nimg * K, device=dev, generator=gen) if rows else None
    dW, db = torch.full((N * K,), float("nan"), device=dev), torch.full((N,), float("nan"), device=dev)
    nw = query("wgrad_workspace_floats", M, N, K)
    call("wgrad_f32", G, N, 0, X, K, 2 if rows else 0, sc, rows if rows else 1, M, N, K, 0, 0, 0, 0, dW, db,
         torch.full((nw,), float("nan"), device=dev), nw, dtype)
    torch.cuda.synchronize()
    Xd = X.double()
    if rows:
        Xd = Xd * sc.view(nimg, K).double().repeat_interleave(rows, 0)[:M]
    _check(dW, db, G.double().t() @ Xd, G.double().sum(0), M)


@pytest.mark.parametrize("B,gh,gw,side", [(2, 32, 32, "x"), (2, 32, 32, "g"), (1, 9, 7, "x"), (3, 5, 11, "g")])
def test_wgrad_full_space_to_depth(dev, B, gh, gw, side):
    """The level-0 / 1 down conv (X = the 2x2 space-to-depth gather of its input, N 64 x K 128) and up conv (G = the
    gather of the PixelShuffle output gradient, N 128 x K 64)."""
    from lowlight_image_enhancement_amd._lib import call, query
    cs, M = 32, B * gh * gw
    gen = torch.Generator(device=dev).manual_seed(M + (side == "g"))
    fmap = torch.randn(B, 2 * gh, 2 * gw, cs, device=dev, generator=gen).to(torch.bfloat16)
    flat = fmap.view(B, gh, 2, gw, 2, cs).permute(0, 1, 3, 2, 4, 5).reshape(M, 4 * cs)  # k = (kh*2 + kw)*cs + c
    other = torch.randn(M, 2 * cs, device=dev, generator=gen).to(torch.bfloat16)
    if side == "x":
        N, K, G, X, gm, xm, csg, csx = 2 * cs, 4 * cs, other, fmap, 0, 1, 0, cs
        ref, bref = other.double().t() @ flat.double(), other.double().sum(0)
    else:
        N, K, G, X, gm, xm, csg, csx = 4 * cs, 2 * cs, fmap, other, 1, 0, cs, 0
        ref, bref = flat.double().t() @ other.double(), flat.double().sum(0)
    dW, db = torch.full((N * K,), float("nan"), device=dev), torch.full((N,), float("nan"), device=dev)
    nw = query("wgrad_workspace_floats", M, N, K)
    call("wgrad_f32", G, N, gm, X, K, xm, None, 1, M, N, K, gh, gw, csg, csx, dW, db,
         torch.full((nw,), float("nan"), device=dev), nw, 1)
    torch.cuda.synchronize()
    _check(dW, db, ref, bref, M)


def test_wgrad_16bit_rejects_misaligned_views(dev):
    """the 16-bit weight-gradient kernels read G and X by 16-byte vectors from the base pointers; a view at
    an odd element offset is refused loudly instead of being read from the wrong addresses."""
    from lowlight_image_enhancement_amd._lib import NBPError, call, query
    M, N, K = 4096, 32, 32
    Gb = torch.zeros(M * N + 8, device=dev, dtype=torch.float16)
    X = torch.zeros(M, K, device=dev, dtype=torch.float16)
    dW, db = torch.empty(N, K, device=dev), torch.empty(N, device=dev)
    n_ws = query("wgrad_workspace_floats", M, N, K)
    ws = torch.empty(n_ws, device=dev)
    call("wgrad_f32", Gb[:M * N].view(M, N), N, 0, X, K, 0, None, 1, M, N, K, 0, 0, 0, 0, dW, db, ws, n_ws, 2)
    with pytest.raises(NBPError, match="16-byte aligned"):
        call("wgrad_f32", Gb[1:1 + M * N].view(M, N), N, 0, X, K, 0, None, 1, M, N, K, 0, 0, 0, 0, dW, db, ws, n_ws, 2)
