"""Cluster-kernel timings for few instances (the latency-bound cases: config 2
and 5, and the tail of a full irl run) across env variants, with bit-identity
checks against the first variant.

usage: python tools/diag/single_bench.py [VARIANT ...]   VARIANT = "ENV=V,ENV=V" (empty: defaults)
env CASES="128x1,64x1,128x4" (grid x instances)
"""
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
variants = sys.argv[1:] or [""]
keys = ("IRLMX_PAIR_NT", "IRLMX_PAIR", "IRLMX_CLUSTER_R", "IRLMX_CLUSTER_G", "IRLMX_SPT_MAX")
cases = [tuple(int(x) for x in c.split("x")) for c in os.environ.get("CASES", "128x1,64x1,128x4").split(",")]
FWD_SWEEPS = int(os.environ.get("FWD_SWEEPS", "60000"))


def h(*ts):
    d = hashlib.sha256()
    for t in ts:
        d.update(t.cpu().numpy().tobytes())
    return d.hexdigest()[:12]


for size, B in cases:
    n = size * size
    mdp = DeviceMDP.icy_gridworld(size, np.linspace(0.1, 0.3, B), device=dev)
    tm = ops.terminal_mask([n - 1], n, batch=B, device=dev)
    r = torch.ones((B, n), dtype=torch.float64, device=dev)
    p0 = torch.zeros((B, n), dtype=torch.float64, device=dev)
    p0[:, 0] = 1.0
    ref = {}
    for v in variants:
        for k in keys:
            os.environ.pop(k, None)
        for kv in filter(None, v.split(",")):
            k, val = kv.split("=")
            os.environ[k] = val
        pb, pf = ops.execution_plan(mdp, "backward"), ops.execution_plan(mdp, "forward")
        pi = ops.backward_maxent(mdp, r, tm)
        torch.cuda.synchronize()
        tb = 1e9
        for _ in range(3):
            t = time.perf_counter(); pi = ops.backward_maxent(mdp, r, tm); torch.cuda.synchronize()
            tb = min(tb, time.perf_counter() - t)
        tf = 1e9
        for _ in range(2):
            t = time.perf_counter(); svf, k, _ = ops.forward_svf(mdp, p0, tm, pi, max_iter=FWD_SWEEPS)
            torch.cuda.synchronize(); tf = min(tf, time.perf_counter() - t)
        kf = int(k.max())
        dig = (h(pi), h(svf, k))
        same = None if not ref else (dig == ref["d"])
        if not ref:
            ref["d"] = dig
        print(f"{size}x{size} B={B} [{v or 'default'}] backward {tb * 1e3:.2f} ms ({tb * 1e6 / (2 * n - 1):.3f} us/sweep; "
              f"R{pb['R']} G{pb['G']} C{pb['C']} spt{pb['spt']} nt{pb['threads']})  forward {tf * 1e3:.2f} ms "
              f"{kf} sweeps ({tf * 1e6 / kf:.3f} us/sweep; R{pf['R']} G{pf['G']} C{pf['C']} spt{pf['spt']} nt{pf['threads']})"
              f"  same as first: {same}", flush=True)
