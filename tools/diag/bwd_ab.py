"""Backward wall time at configs 3 and 4 (128x128 B = 64, 256x256 B = 32, the
bench's slips and theta = 1) for A/B of library builds (IRLMX_LIB=<path>,
tools/diag/build_variant.sh).  usage: IRLMX_LIB=... python tools/diag/bwd_ab.py [tag]"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import torch
from irlmx import DeviceMDP, ops
from irlmx.shard import instance_slips
dev = torch.device("cuda", 0)
tag = sys.argv[1] if len(sys.argv) > 1 else os.environ.get("IRLMX_LIB", "default")
out = []
for size, B, reps in ((128, 64, 5), (256, 32, 2)):
    n = size * size
    mdp = DeviceMDP.icy_gridworld(size, instance_slips(np.arange(B), B), device=dev)
    tm = ops.terminal_mask([n - 1], n, batch=B, device=dev)
    r = torch.ones((B, n), dtype=torch.float64, device=dev)
    ops.backward_maxent(mdp, r, tm)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        ops.backward_maxent(mdp, r, tm)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
    out.append(f"{size}x{size} B={B}: backward {np.median(ts):.2f} ms (min {min(ts):.2f})")
    del mdp, tm, r
    torch.cuda.empty_cache()
print(f"[{tag}] " + " | ".join(out), flush=True)
