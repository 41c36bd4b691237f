"""world_size-2 gloo rehearsal of the multi-GPU bench path on CPU.

Frames shard across ranks with no data-path collective; ranks meet only at the
barrier and at the max-over-ranks of the timed region (orb_slam2_commit_amd/dist.py)."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    from orb_slam2_commit_amd import dist as odist
    import torch.distributed as dist
    odist.init("gloo", rank, world)
    odist.barrier()
    elapsed = 1.0 + rank  # rank 1 is the slow one
    m = odist.max_over_ranks(elapsed)
    seeds = odist.frame_seeds(rank, 4)
    its = odist.sum_over_ranks(15.0 + rank)  # LocalBA leg: iterations summed over ranks
    q.put((rank, m, seeds, odist.job_throughput(8, 10, world, m), its))
    dist.destroy_process_group()


def test_gloo_world2_max_and_shards():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[1] == 2.0 for r in res)  # max over ranks
    assert set(res[0][2]).isdisjoint(res[1][2])  # disjoint frame shards
    assert res[0][3] == pytest.approx(8 * 10 * 2 / 2.0)
    assert all(r[4] == 31.0 for r in res)


def test_single_rank_noop():
    from orb_slam2_commit_amd import dist as odist
    assert odist.max_over_ranks(3.5) == 3.5
    assert odist.sum_over_ranks(3.5) == 3.5
    assert odist.job_throughput(128, 20, 1, 2.0) == 1280.0


# ------------------------------------------------------------------ bench.py --gpus launcher
def _bench():
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m, root


def test_bench_rank_plan_and_launcher_cmd():
    import argparse
    b, root = _bench()
    a = argparse.Namespace(gpus=1)
    assert b.rank_plan(a, env={}) == ("rank", 1)
    a.gpus = 8
    assert b.rank_plan(a, env={}) == ("launch", 8)  # plain `bench.py --gpus 8`: launch 8 ranks
    assert b.rank_plan(a, env={"WORLD_SIZE": "8"}) == ("rank", 8)
    with pytest.raises(SystemExit, match="WORLD_SIZE=1 but --gpus 8"):
        b.rank_plan(a, env={"WORLD_SIZE": "1"})
    with pytest.raises(SystemExit):
        b.rank_plan(argparse.Namespace(gpus=0), env={})
    cmd = b.launcher_cmd(4, ["--gpus", "4", "--steps", "5"], 29600)
    i = cmd.index("torch.distributed.run")
    assert cmd[i - 1] == "-m" and cmd[0]
    assert cmd[i + 1:i + 10] == ["--nnodes=1", "--nproc-per-node", "4", "--master-addr", "127.0.0.1",
                                 "--master-port", "29600", os.path.join(root, "bench.py"), "--gpus"]
    assert cmd[-4:] == ["--gpus", "4", "--steps", "5"]  # the ranks get the same arguments


def test_bench_world_size_mismatch_fails_loudly():
    """A rank started with WORLD_SIZE != --gpus exits non-zero before touching torch."""
    import subprocess
    import sys
    _, root = _bench()
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=2 but --gpus 4" in r.stderr


def test_bench_launcher_refuses_more_ranks_than_gpus_under_rccl():
    import subprocess
    import sys
    import torch
    _, root = _bench()
    n = max(2, torch.cuda.device_count() + 1)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["ORBX_DIST_BACKEND"] = "nccl"
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(n)], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "GPU(s) visible" in r.stderr
