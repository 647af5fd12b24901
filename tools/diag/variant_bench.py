"""Cluster-kernel timings for comparing library builds (IRLMX_LIB=build/<name>/libirlmx.so,
tools/diag/build_variant.sh): config 3 backward + forward (128x128, B = 64, theta = 1), config 4
backward (256x256, B = 32) and one 128x128 instance's forward, each the minimum of 3 calls, plus a
digest of every result so that variants can be checked for bit identity."""
import hashlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import torch  # noqa: E402
from irlmx import DeviceMDP, ops  # noqa: E402

dev = torch.device("cuda", 0)
which = os.environ.get("WHICH", "c3b,c3f,c4b,c1f").split(",")
label = os.environ.get("IRLMX_LIB", "in-tree")


def digest(*ts):
    h = hashlib.sha256()
    for t in ts:
        h.update(t.detach().cpu().numpy().tobytes())
    return h.hexdigest()[:12]


def timed(fn, n=3):
    out = fn(); torch.cuda.synchronize()
    best = 1e9
    for _ in range(n):
        t = time.perf_counter(); out = fn(); torch.cuda.synchronize(); best = min(best, time.perf_counter() - t)
    return best * 1e3, out


def case(size, B):
    n = size * size
    mdp = DeviceMDP.icy_gridworld(size, np.linspace(0.1, 0.3, B), device=dev)
    tm = ops.terminal_mask([n - 1], n, batch=B, device=dev)
    r = torch.ones((B, n), dtype=torch.float64, device=dev)
    p0 = torch.zeros((B, n), dtype=torch.float64, device=dev); p0[:, 0] = 1.0
    return mdp, tm, r, p0


if "c3b" in which or "c3f" in which:
    mdp, tm, r, p0 = case(128, 64)
    tb, pi = timed(lambda: ops.backward_maxent(mdp, r, tm))
    print(f"[{label}] c3 backward {tb:.2f} ms  digest {digest(pi)}", flush=True)
    if "c3f" in which:
        tf, (svf, k, _) = timed(lambda: ops.forward_svf(mdp, p0, tm, pi, max_iter=400000), n=1)
        print(f"[{label}] c3 forward(theta=1) {tf:.2f} ms sweeps {int(k.max())}  digest {digest(svf, k)}", flush=True)
if "c4b" in which:
    mdp, tm, r, p0 = case(256, 32)
    tb, pi = timed(lambda: ops.backward_maxent(mdp, r, tm), n=2)
    print(f"[{label}] c4 backward {tb:.2f} ms  digest {digest(pi)}", flush=True)
if "c1f" in which:
    mdp, tm, r, p0 = case(128, 1)
    pi = ops.backward_maxent(mdp, r, tm)
    tf, (svf, k, _) = timed(lambda: ops.forward_svf(mdp, p0, tm, pi, max_iter=400000), n=2)
    print(f"[{label}] 128x128 x1 forward {tf:.2f} ms sweeps {int(k.max())} ({tf * 1e3 / int(k.max()):.3f} us/sweep)"
          f"  digest {digest(svf, k)}", flush=True)
