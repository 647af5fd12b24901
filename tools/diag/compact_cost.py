"""First-use cost of the pieces of BatchedMaxEnt.compact() / update() on the
working set (the full run's outlier steps): each statement timed with a sync,
for working batches 62, 17, 16, 15, 1 in a fresh process, twice.
usage: python tools/diag/compact_cost.py"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import torch
from irlmx import DeviceMDP, ops
from irlmx.shard import instance_slips

dev = torch.device("cuda", 0)
B, size = 64, 128
S = size * size
mdp = DeviceMDP.icy_gridworld(size, instance_slips(np.arange(B), B), device=dev)
e_f = torch.zeros((B, S), dtype=torch.float64, device=dev)
term = ops.terminal_mask([S - 1], S, batch=B, device=dev)
theta = torch.ones((B, S), dtype=torch.float64, device=dev)
torch.cuda.synchronize()


def timed(name, fn):
    torch.cuda.synchronize()
    t = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) * 1e3
    print(f"    {name:28s} {dt:9.3f} ms", flush=True)
    return r


for rep in range(2):
    for n in (62, 17, 16, 15, 1):
        print(f"rep {rep} working batch {n}", flush=True)
        active = torch.zeros(B, dtype=torch.bool, device=dev)
        active[:n] = True
        idx = timed("nonzero", lambda: torch.nonzero(active).squeeze(1))
        timed("int(numel)", lambda: int(idx.numel()))
        timed("take(row_val f64 4D)", lambda: mdp.take(idx))
        timed("index_select e_f f64", lambda: e_f.index_select(0, idx).contiguous())
        timed("index_select term u8", lambda: term.index_select(0, idx).contiguous())
        timed("ones bool", lambda: torch.ones(n, dtype=torch.bool, device=dev))
        th = timed("index_select theta", lambda: theta.index_select(0, idx))
        act = timed("index_select active bool", lambda: active.index_select(0, idx))
        new = timed("exp-sga", lambda: th * torch.exp(0.1 * (e_f[:n] - th)))
        d = timed("where/amax", lambda: torch.where(act, (new - th).abs().amax(dim=1),
                                                    torch.zeros((), dtype=torch.float64, device=dev)))
        timed("index_put theta", lambda: theta.__setitem__(idx, new))
        timed("scatter (full + index_put)", lambda: torch.full((B,), 0, dtype=d.dtype, device=dev).__setitem__(idx, d))
        timed("scatter int64", lambda: torch.full((B,), 0, dtype=torch.int64, device=dev).__setitem__(
            idx, torch.zeros(n, dtype=torch.int64, device=dev)))
        timed("active &= gt", lambda: active.__iand__(torch.zeros(B, dtype=torch.float64, device=dev) > 1e-4))
