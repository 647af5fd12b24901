"""Multi-process paths of the instance sharding (gloo, world sizes 2, 4 and 8).

CPU: shard ranges cover every instance exactly once; the timing max-reduction
and the result gather work over gloo.  GPU: two ranks share cuda:0 and each
runs its block of instances; the gathered result equals one process running
the whole batch bit for bit (instances are independent; no data-path
collective).
"""

import os
import socket
import subprocess
import sys
import textwrap

import numpy as np
import pytest

from conftest import PKG_DIR, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_shard_ranges_cover_all():
    from irlmx.shard import shard_range
    for n in (1, 7, 64, 256):
        for world in (1, 2, 3, 8):
            got = []
            for r in range(world):
                lo, hi = shard_range(n, world, r)
                got.extend(range(lo, hi))
            assert got == list(range(n))


WORKER = textwrap.dedent("""
    import os, sys, json
    sys.path.insert(0, {pkg!r})
    import numpy as np, torch, torch.distributed as dist
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:{port}", rank={rank}, world_size=2)
    from irlmx.shard import shard_range, max_over_ranks, gather_to_rank0
    rank = dist.get_rank()
    lo, hi = shard_range(9, 2, rank)
    t = max_over_ranks(1.0 + rank)
    mode = {mode!r}
    if mode == "cpu":
        local = torch.arange(lo, hi, dtype=torch.float64)[:, None] * torch.ones(1, 3, dtype=torch.float64)
    else:
        from irlmx import DeviceMDP, ops
        from irlmx.shard import instance_slips
        dev = torch.device("cuda", 0)
        size = 6; n = size * size
        mdp = DeviceMDP.icy_gridworld(size, instance_slips(np.arange(lo, hi), 9), device=dev)
        rew = np.random.default_rng(5).uniform(0, 1, (9, n))[lo:hi]
        tm = ops.terminal_mask([n - 1], n, batch=hi - lo, device=dev)
        pi = ops.backward_maxent(mdp, rew, tm)
        p0 = np.zeros((hi - lo, n)); p0[:, 0] = 1.0
        svf, k, _ = ops.forward_svf(mdp, p0, tm, pi)
        local = svf
    out = gather_to_rank0(local, 9)
    if rank == 0:
        np.save({out!r}, out.numpy())
        json.dump({{"tmax": t}}, open({out!r} + ".json", "w"))
    dist.destroy_process_group()
""")


def _run_pair(tmp_path, mode):
    port = _free_port()
    out = str(tmp_path / f"gathered_{mode}.npy")
    procs = []
    for rank in range(2):
        code = WORKER.format(pkg=PKG_DIR, port=port, rank=rank, mode=mode, out=out)
        env = dict(os.environ, MASTER_ADDR="127.0.0.1")
        procs.append(subprocess.Popen([sys.executable, "-c", code], env=env, cwd=ROOT))
    for p in procs:
        assert p.wait(timeout=240) == 0
    import json
    return np.load(out), json.load(open(out + ".json"))


BENCH_WORKER = textwrap.dedent("""
    import json, os, sys, time
    sys.path[:0] = [{root!r}, {pkg!r}]
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:{port}", rank={rank}, world_size={world})
    import bench
    from irlmx.shard import instance_slips, max_over_ranks, shard_range
    rank, world, per_gpu = dist.get_rank(), {world}, {per_gpu}
    lo, hi = shard_range(per_gpu * world, world, rank)
    done = []
    def step(i, timed):  # stub: rank 1 is the slow rank
        done.append((i, timed))
        time.sleep(0.02 * (rank + 1))
    elapsed, per_step = bench.timed_steps(step, 3, 1, dist.barrier, lambda: None)
    emax = max_over_ranks(elapsed)
    value, ms = bench.headline(emax, per_gpu, world, 3)
    json.dump({{"rank": rank, "lo": lo, "hi": hi, "slips": instance_slips(range(lo, hi), per_gpu * world).tolist(),
               "elapsed": elapsed, "emax": emax, "value": value, "ms": ms, "done": done,
               "device": bench.rank_device({rank}, 8)}},
              open({out!r} + f".{{rank}}.json", "w"))
    dist.destroy_process_group()
""")


@pytest.mark.parametrize("world,per_gpu", [(2, 4), (4, 4), (8, 32)])
def test_bench_timing_over_gloo(tmp_path, world, per_gpu):
    """bench.py's multi-rank arithmetic with a stubbed step (gloo; 2 and 4 ranks,
    and config 4's layout: 8 ranks x 32 instances = the 256-instance batch):
    each rank times exactly K steps after W warm-ups between barriers, the elapsed
    time is the max over ranks, value = instances on all ranks x K / that max, the
    shards cover the global batch with the bench's per-instance slips, and every
    rank of an 8-GPU node gets its own device."""
    import json
    port = _free_port()
    out = str(tmp_path / "bench")
    procs = [subprocess.Popen([sys.executable, "-c", BENCH_WORKER.format(root=ROOT, pkg=PKG_DIR, port=port, rank=r,
                                                                          out=out, world=world, per_gpu=per_gpu)],
                              cwd=ROOT)
             for r in range(world)]
    for p in procs:
        assert p.wait(timeout=240) == 0
    res = [json.load(open(f"{out}.{r}.json")) for r in range(world)]
    assert all(r["emax"] == max(x["elapsed"] for x in res) for r in res)
    assert res[-1]["elapsed"] >= 3 * 0.02 * world
    for r in res:
        assert r["value"] == per_gpu * world * 3 / r["emax"] and abs(r["ms"] - r["emax"] / 3 * 1e3) < 1e-9
        assert r["done"] == [[0, False], [1, True], [2, True], [3, True]]
    assert [(r["lo"], r["hi"]) for r in res] == [(per_gpu * k, per_gpu * k + per_gpu) for k in range(world)]
    B = per_gpu * world
    assert sum((r["slips"] for r in res), []) == [0.1 + 0.2 * b / B for b in range(B)]
    assert sorted(r["device"] for r in res) == list(range(world))   # one distinct GPU per rank


def test_rank_device_mapping():
    """bench.py's LOCAL_RANK -> device choice: one GPU per rank on a full node;
    more ranks than GPUs (a rehearsal on a 1-GPU box) share them round-robin."""
    import bench
    assert [bench.rank_device(r, 8) for r in range(8)] == list(range(8))
    assert [bench.rank_device(r, 1) for r in range(4)] == [0, 0, 0, 0]
    assert [bench.rank_device(r, 2) for r in range(4)] == [0, 1, 0, 1]
    assert bench.rank_device(3, 0) == 0


def test_gloo_gather_and_max(tmp_path):
    got, meta = _run_pair(tmp_path, "cpu")
    assert meta["tmax"] == 2.0
    assert np.array_equal(got, np.arange(9.0)[:, None] * np.ones((1, 3)))


@pytest.mark.gpu
def test_sharded_equals_single_process(tmp_path):
    import torch
    import __graft_entry__ as g
    g.build()
    from irlmx import DeviceMDP, ops
    from irlmx.shard import instance_slips
    got, _ = _run_pair(tmp_path, "gpu")
    dev = torch.device("cuda", 0)
    size, n = 6, 36
    mdp = DeviceMDP.icy_gridworld(size, instance_slips(np.arange(9), 9), device=dev)
    rew = np.random.default_rng(5).uniform(0, 1, (9, n))
    tm = ops.terminal_mask([n - 1], n, batch=9, device=dev)
    pi = ops.backward_maxent(mdp, rew, tm)
    p0 = np.zeros((9, n))
    p0[:, 0] = 1.0
    svf, _, _ = ops.forward_svf(mdp, p0, tm, pi)
    assert np.array_equal(got, svf.cpu().numpy())
