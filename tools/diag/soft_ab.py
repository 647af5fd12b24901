"""Soft VI wall time per call for A/B of library builds (IRLMX_LIB=<path>):
config 5's 128x128 (one instance and 64 instances, the bench's slips and
theta = 1, discount 0.7) and config 2's 64x64 in numpy's order (the drop-in's
default there).  usage: [IRLMX_LIB=...] python tools/diag/soft_ab.py [tag]"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import torch
from irlmx import DeviceMDP, ops
from irlmx.batch import terminal_reward
from irlmx.shard import instance_slips
dev = torch.device("cuda", 0)
tag = sys.argv[1] if len(sys.argv) > 1 else os.environ.get("IRLMX_LIB", "default")
out = []
for size, B, npo, reps in ((128, 1, False, 5), (128, 64, False, 3), (64, 1, True, 3)):
    n = size * size
    slips = 0.2 if B == 1 else instance_slips(np.arange(B), B)
    mdp = DeviceMDP.icy_gridworld(size, slips, device=dev)
    r = torch.ones((B, n), dtype=torch.float64, device=dev)
    phi = terminal_reward([n - 1], n, B, dev)
    ops.soft_backward(mdp, r, phi, 0.7, numpy_order=npo)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        _, _, k, _ = ops.soft_backward(mdp, r, phi, 0.7, numpy_order=npo)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
    out.append(f"{size}x{size} B={B}{' numpy-order' if npo else ''}: {np.median(ts):.2f} ms ({int(k.max())} sweeps)")
print(f"[{tag}] " + " | ".join(out), flush=True)
