"""One flush of many deferred gradient reductions (more than one by-value batch: the device descriptor table and ONE
reduce_table_kernel launch, gemm.hip launch_multi) against the same reductions launched one at a time (immediate mode,
reduce_multi_kernel with one descriptor): bitwise equal -- every descriptor runs the same reduction code in both -- and
against a float64 column sum.  The flush also carries layer-scale post-ops whose U / V are reductions of the same flush
(the table's row descriptors, U / V never written): against float64 (the immediate path reduces U / V with other
row-lane splits, so those are not bitwise comparable)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _problems(dev, n, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    out = []
    for i in range(n):
        S = int(torch.randint(1, 300, (1,), generator=g, device=dev))
        L = int(torch.randint(1, 3000, (1,), generator=g, device=dev)) * (4 if i % 3 else 1) + (i % 2)
        out.append(torch.randn(S, L, device=dev, generator=g))
    return out


def _layer_scale(dev, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    N, K, S = 64, 128, 37
    R = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa: E731
    return dict(slabU=R(S, N * K), slabV=R(S, N), W=R(N, K), b=R(N), scale=R(N), N=N, K=K, S=S)


def _run(dev, slabs, ls, deferred):
    from lowlight_image_enhancement_amd._lib import call
    outs = [torch.full((s.shape[1],), float("nan"), device=dev) for s in slabs]
    lo = []
    if deferred:
        call("grad_reduce_defer")
    for s, o in zip(slabs, outs):
        call("reduce_slab", s, s.shape[0], s.shape[1], o)
    for d in ls:
        U, V = torch.empty(d["N"] * d["K"], device=dev), torch.empty(d["N"], device=dev)
        dW, db, ds = (torch.full((n,), float("nan"), device=dev) for n in (d["N"] * d["K"], d["N"], d["N"]))
        call("reduce_slab", d["slabU"], d["S"], d["N"] * d["K"], U)
        call("reduce_slab", d["slabV"], d["S"], d["N"], V)
        call("layer_scale_grad", U, V, d["W"], d["b"], d["scale"], dW, db, ds, d["N"], d["K"])
        lo.append((dW, db, ds))
    if deferred:
        call("grad_reduce_flush", 1)
    torch.cuda.synchronize()
    return outs, lo


def test_flush_table_bitwise_equals_immediate(dev):
    from lowlight_image_enhancement_amd._lib import last_call_stats
    slabs = _problems(dev, 100, 5)
    ls = [_layer_scale(dev, 9 + k) for k in range(10)]
    got, glo = _run(dev, slabs, ls, True)
    st = last_call_stats(1)
    ref, _ = _run(dev, slabs, [], False)
    assert st[3] == 1, st  # the whole flush (100 slabs, 10 layer-scale row sets) as one reduction launch
    for a, b in zip(got, ref):
        assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    for s, a in zip(slabs, got):
        r = s.double().sum(0)
        assert (a.double() - r).abs().max().item() <= 1e-5 * (1 + r.abs().max().item())
    for d, (dW, db, ds) in zip(ls, glo):
        U = d["slabU"].double().sum(0).view(d["N"], d["K"])
        V = d["slabV"].double().sum(0)
        sc = d["scale"].double()
        for x, r in ((dW, (sc[:, None] * U).flatten()), (db, sc * V),
                     (ds, (d["W"].double() * U).sum(1) + d["b"].double() * V)):
            assert (x.double() - r).abs().max().item() <= 1e-4 * (1 + r.abs().max().item())
