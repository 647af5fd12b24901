"""Persistent shapes when their workgroups cannot all run at once (needs an MI355X).

The cluster and grid shapes hand data between workgroups inside one launch,
so they need every workgroup of the launch resident together.  When another
kernel or process holds CUs that is not the case; each launch therefore starts
with a two-phase rendezvous (cluster.h ``coresident``) and, if it fails, the
call is rerun on the per-sweep shape -- same arithmetic, bit-identical results
(maxent.py:107-112, 154-156, 326-338; solver.py:40-50).

* ``IRLMX_TEST_NOT_RESIDENT=1`` makes every persistent launch wait for one
  workgroup more than it has, i.e. take the fallback deterministically: results
  must equal the normal run bit for bit.
* Two host threads, and two processes, running the config-3 backward (256
  persistent workgroups each, one per CU) at the same time on one GPU: every
  result bit-identical to a lone call, no exchange timeout.
"""

import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dev():
    import __graft_entry__ as g
    g.build()
    import irlmx
    return irlmx.require_device()


def _bits(x):
    return x.view(torch.int64) if x.dtype == torch.float64 else x


def _same(a, b):
    flat = lambda t: list(t) if isinstance(t, tuple) else [t]
    for x, y in zip(flat(a), flat(b)):
        assert torch.equal(_bits(x), _bits(y))


def test_not_resident_fallback_is_bit_identical(dev, monkeypatch):
    from irlmx import DeviceMDP, ops
    from irlmx.batch import terminal_reward
    size, n = 128, 128 * 128
    mdp = DeviceMDP.icy_gridworld(size, [0.1, 0.3], device=dev)
    assert ops.execution_plan(mdp, "backward")["shape"] == "cluster"
    assert ops.execution_plan(mdp, "soft_backward")["shape"] == "grid"
    rng = np.random.default_rng(7)
    r = rng.uniform(0.0, 1.0, (2, n))
    tm = ops.terminal_mask([n - 1], n, batch=2, device=dev)
    p0 = np.zeros((2, n))
    p0[:, 0] = 1.0
    phi = terminal_reward([n - 1], n, 2, dev)

    def run():
        pi = ops.backward_maxent(mdp, r, tm)
        return (pi, ops.forward_svf(mdp, p0, tm, pi, max_iter=2000), ops.soft_backward(mdp, r, phi, 0.7),
                ops.value_iteration(mdp, r, 0.9))

    ref = run()
    monkeypatch.setenv("IRLMX_TEST_NOT_RESIDENT", "1")
    got = run()
    for g_, r_ in zip(got, ref):
        _same(g_, r_)


def test_two_streams_at_once(dev):
    """Two host threads run config 3's backward (256 workgroups, one full CU
    each) on two streams at the same time: the two launches compete for the
    CUs, so at most one can have all its workgroups resident.  Both calls must
    finish, bit-identical to a lone call (the loser falls back after the
    rendezvous instead of spinning into the exchange timeout)."""
    import threading
    from irlmx import DeviceMDP, ops
    n = 128 * 128
    mdp = DeviceMDP.icy_gridworld(128, np.linspace(0.1, 0.3, 64), device=dev)
    plan = ops.execution_plan(mdp, "backward")
    assert plan["shape"] == "cluster" and plan["C"] * plan["per_launch"] == 256
    tm = ops.terminal_mask([n - 1], n, batch=64, device=dev)
    r = torch.ones((64, n), dtype=torch.float64, device=dev)
    ref = ops.backward_maxent(mdp, r, tm)
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    out, errs = [[], []], []

    def worker(k):
        try:
            with torch.cuda.stream(streams[k]):
                for _ in range(4):
                    out[k].append(ops.backward_maxent(mdp, r, tm))
                streams[k].synchronize()
        except Exception as e:  # surfaced below
            errs.append(repr(e))

    threads = [threading.Thread(target=worker, args=(k,)) for k in range(2)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=200)
    assert not errs, errs
    assert len(out[0]) == len(out[1]) == 4
    for got in out[0] + out[1]:
        assert torch.equal(_bits(got), _bits(ref))


_CHILD = r"""
import hashlib, os, sys
sys.path[:0] = [os.path.join(os.environ["ROOT"], "irl-maxent_amd")]
import numpy as np, torch
from irlmx import DeviceMDP, ops
dev = torch.device("cuda", 0)
n = 128 * 128
mdp = DeviceMDP.icy_gridworld(128, np.linspace(0.1, 0.3, 64), device=dev)
tm = ops.terminal_mask([n - 1], n, batch=64, device=dev)
r = torch.ones((64, n), dtype=torch.float64, device=dev)
for _ in range(int(os.environ["REPS"])):
    pi = ops.backward_maxent(mdp, r, tm)
    torch.cuda.synchronize()
    print(hashlib.sha256(pi.cpu().numpy().tobytes()).hexdigest(), flush=True)
"""


def test_two_processes_share_the_gpu(dev):
    env = dict(os.environ, ROOT=ROOT, REPS="12")
    env.pop("IRLMX_TEST_NOT_RESIDENT", None)
    procs = [subprocess.Popen([sys.executable, "-c", _CHILD], env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for _ in range(2)]
    outs = []
    for p in procs:
        out, err = p.communicate(timeout=240)
        assert p.returncode == 0, err[-2000:]
        outs.append(out.split())
    digests = set(outs[0]) | set(outs[1])
    assert len(outs[0]) == len(outs[1]) == 12
    assert len(digests) == 1, digests
