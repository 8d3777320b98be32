"""bench.py --gpus N argument handling (CPU): N ranks are started (or required from the launcher) exactly as asked,
never silently one.  The launch contract mirrors the reference's DDP launch
(NAFNet_base/basicsr/train.py:54-63, utils/dist_util.py:28-40): one process per GPU, RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT in the environment."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_plan_single_gpu_default():
    assert bench.plan_launch(None, {}, 1, False) == ("run", 1)
    assert bench.plan_launch(1, {}, 8, False) == ("run", 1)


def test_plan_spawns_n_ranks_without_a_launcher():
    assert bench.plan_launch(8, {}, 8, False) == ("spawn", 8)
    assert bench.plan_launch(2, {}, 1, True) == ("spawn", 2)  # rehearsal: every rank on cuda:0


def test_plan_under_a_launcher_must_match():
    assert bench.plan_launch(4, {"WORLD_SIZE": "4"}, 8, False) == ("run", 4)
    assert bench.plan_launch(None, {"WORLD_SIZE": "2"}, 8, False) == ("run", 2)
    with pytest.raises(SystemExit, match="must match"):
        bench.plan_launch(8, {"WORLD_SIZE": "1"}, 8, False)


def test_plan_refuses_more_ranks_than_gpus():
    with pytest.raises(SystemExit, match="only 1 GPU"):
        bench.plan_launch(8, {}, 1, False)
    with pytest.raises(SystemExit, match=">= 1"):
        bench.plan_launch(0, {}, 8, False)


def test_rank_envs_are_torchrun_style():
    envs = bench.rank_envs(4, {"FOO": "1"}, 29555)
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    for e in envs:
        assert e["WORLD_SIZE"] == "4" and e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29555"
        assert e["FOO"] == "1"


def _run(args, env_extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=300)


def test_mismatched_world_size_exits_nonzero():
    r = _run(["--gpus", "2"], {"WORLD_SIZE": "3"})
    assert r.returncode != 0 and "must match" in r.stderr


def test_spawned_ranks_report_their_failure():
    """Stand-alone --gpus 2 (rehearsal, so the GPU count check passes here): the parent starts two ranks with
    WORLD_SIZE=2; on this GPU-less container each rank fails at its first GPU call, and the parent exits non-zero
    instead of timing one process."""
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--quick"], {"NBP_BENCH_REHEARSE": "1"})
    assert r.returncode != 0
    assert "exited with status" in r.stderr
    assert '"n_gpus"' not in r.stdout


@pytest.mark.gpu
def test_rehearsal_line_carries_the_comm_fields():
    """The N > 1 bench line, rehearsed on the one-GPU box: two ranks on cuda:0 over gloo run the
    graph segments and bucket all-reduces; rank 0's JSON line reports the buckets and bytes all-reduced per step, the
    exposed all-reduce time of graph replays and of the eager steps, and the NAFBlock figure net of that time."""
    import json
    r = _run(["--gpus", "2", "--steps", "3", "--warmup", "1", "--quick"], {"NBP_BENCH_REHEARSE": "1"})
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["rehearsal"]
    c = line["comm"]
    assert c["buckets_per_step"] >= 1 and c["bytes_allreduced_per_step"] == 4 * 29159715
    assert c["allreduce_exposed_ms"] is not None and c["allreduce_exposed_ms"] >= 0
    assert c["allreduce_exposed_ms_eager"] is not None and c["probed_steps"] >= 1
    assert "exposed all-reduce" in line["nafblock_roofline"]["ms_method"]


def _newest_kernel_stats():
    import glob
    fs = [f for f in glob.glob(os.path.join(ROOT, "profiles", "*", "kernel_stats.csv"))]
    key = lambda f: bench._pmc_newest_key(f)  # noqa: E731
    return sorted(fs, key=key)[-1] if fs else None


def test_single_kernel_classes_name_one_rocprof_instance():
    """every one-instance class of the bench (the candidates for the headline `roofline`) names
    exactly one kernel instance per storage type in the newest committed rocprof summary (or none, if the record's
    step never launched it), and the launch records the library writes map onto those classes."""
    import csv
    import re
    path = _newest_kernel_stats()
    assert path is not None
    names = [r["Name"] for r in csv.DictReader(open(path))]
    # the record's own bench line: a class it saw launched must name exactly one instance (a template parameter added
    # to a kernel changes its mangled name: a stale regex would otherwise match nothing, silently)
    bj = os.path.join(os.path.dirname(path), "bench.json")
    launched = set()
    if os.path.exists(bj):
        import json
        classes = json.load(open(bj))["roofline"].get("classes", {})
        launched = {c for c, v in classes.items() if (v.get("launches_per_step") or 0) > 0}
    seen = 0
    for cls in bench.SINGLE_KERNEL:
        pats = [re.compile(p.format(T=bench.MANGLED_T["fp16"])) for p in bench.ROCPROF_KERNELS[cls]]
        hits = [n for n in names if any(p.search(n) for p in pats)]
        assert len(hits) <= 1, (cls, hits)
        if cls in launched:
            assert len(hits) == 1, (cls, "launched in the record's bench line but no rocprof instance matches")
        seen += len(hits)
    assert seen >= 5, path
    # the instance names the library records (nbp_launch_timing) are the keys of bench.INSTANCES
    src = "".join(open(os.path.join(ROOT, "lowlight_image_enhancement_amd", "csrc", f)).read()
                  for f in ("gemm.hip", "dwconv.hip", "c1dw_tile.hip", "ffn_rows.hip"))
    for inst in bench.INSTANCES:
        assert f'"{inst}"' in src, inst
