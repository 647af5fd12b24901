"""Wall time of the cluster passes the bench configs run, for A/B of library
builds (IRLMX_LIB=<path> loads a variant, tools/diag/build_variant.sh):
config 3's backward (128x128, B = 64) and a 3,000-sweep forward, one 128x128
instance's 20,000-sweep forward (config 5's shape) and config 2's backward
(64x64 solo).  usage: IRLMX_LIB=... python tools/diag/ab_passes.py [tag]"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import torch
from irlmx import DeviceMDP, ops
from irlmx.shard import instance_slips
dev = torch.device("cuda", 0)
tag = sys.argv[1] if len(sys.argv) > 1 else os.environ.get("IRLMX_LIB", "default")


def timed(fn, reps=3):
    fn(); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


out = []
for size, B, fwd_cap in ((128, 64, 3000), (128, 1, 20000), (64, 1, 0)):
    n = size * size
    mdp = DeviceMDP.icy_gridworld(size, instance_slips(np.arange(B), B), device=dev)
    tm = ops.terminal_mask([n - 1], n, batch=B, device=dev)
    r = torch.ones((B, n), dtype=torch.float64, device=dev)
    p0 = torch.zeros((B, n), dtype=torch.float64, device=dev)
    p0[:, 0] = 1.0
    tb = timed(lambda: ops.backward_maxent(mdp, r, tm))
    pi = ops.backward_maxent(mdp, r, tm)
    tf = timed(lambda: ops.forward_svf(mdp, p0, tm, pi, max_iter=fwd_cap)) if fwd_cap else float("nan")
    out.append(f"{size}x{size} B={B}: backward {tb:.3f} ms, forward({fwd_cap}) {tf:.3f} ms")
print(f"[{tag}] " + " | ".join(out), flush=True)
