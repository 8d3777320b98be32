"""RCCL on the trainer's data-parallel path (reference contract: the DDP gradient all-reduce of
base_model.py:72-78 / NAFNet_base/basicsr/train.py:54-63).

The box has one GPU, so the 'nccl' backend (RCCL on ROCm) runs as a ONE-rank process group: the trainer is forced onto
the bucketed path (`data_parallel=True`: per-stage hooks, asynchronous bucket all-reduces through RCCL during the
backward, graph segments cut at the buckets with the all-reduces launched between the replays) and must give bitwise
the parameters, gradients and losses of the plain step -- a one-rank SUM all-reduce is the identity.  The worker is a
fresh spawned process (no exec), so the RCCL library is loaded there and nowhere else; it reports whether librccl is
mapped."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CFG = dict(width=32, enc_blk_nums=[1, 1, 1], middle_blk_num=1, dec_blk_nums=[1, 1, 1])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(dp, graph, precision):
    from lowlight_image_enhancement_amd.NewBP_model.newbp_net_arch import create_newbp_net
    from lowlight_image_enhancement_amd.train import NBPTrainer
    torch.manual_seed(0)
    net = create_newbp_net(in_channels=3, kernel_type="rgb", kernel_spec="B2", **CFG)
    with torch.no_grad():
        net.flat.add_(torch.randn_like(net.flat) * 0.05)
    net = net.cuda()
    net.precision = precision
    # 0.05 MB buckets: several buckets, segments and all-reduces per step
    tr = NBPTrainer(net, psf_mode="rgb", psf_spec="B2", w_l1=1.0, w_ssim=0.05, w_phys=0.1, bucket_mb=0.05,
                    data_parallel=dp)
    fn = tr.graph_step if graph else tr.step
    for s in range(3):
        g = torch.Generator(device="cuda").manual_seed(100 + s)
        lq, gt = (torch.rand(2, 3, 64, 64, device="cuda", generator=g) for _ in range(2))
        fn(lq, gt, lq.clamp(0, 1), torch.ones(2, 1, 1, 1, device="cuda"))
    torch.cuda.synchronize()
    return (tr.net.flat.detach().cpu().numpy().copy(), tr.grad.cpu().numpy().copy(), tr.logs()["Total"],
            len(tr.comm_buckets), len(getattr(tr, "_segs", None) or []))


def _worker(port, precision, q):
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        res = {(dp, graph): _run(dp, graph, precision) for dp in (True, False) for graph in (False, True)}
        maps = open("/proc/self/maps").read()
        q.put((res, "librccl" in maps))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("precision", ["fp32", "fp16"])
def test_rccl_one_rank_bucketed_step_bitwise_equals_plain_step(precision):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    env_ipc = os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")
    assert env_ipc in (None, "0"), "dmabuf IPC mode expected on this pool"
    p = ctx.Process(target=_worker, args=(_free_port(), precision, q))
    p.start()
    res, rccl_mapped = q.get(timeout=300)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert rccl_mapped, "librccl was not loaded by the nccl process group"
    for graph in (False, True):
        pd, gd, ld, nb, nseg = res[(True, graph)]
        p0, g0, l0, nb0, _ = res[(False, graph)]
        assert nb >= 3, nb  # the bucketed path ran: several RCCL all-reduces per step
        assert nb0 == 0
        if graph:
            assert nseg >= 3, nseg  # graph segments cut at the buckets
        assert np.array_equal(pd, p0), graph
        assert np.array_equal(gd, g0), graph
        assert ld == l0, graph
