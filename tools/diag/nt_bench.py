"""Backward cluster-kernel timing at config 3 (128x128, 64 instances) across
workgroup sizes / layouts / plans (env overrides), with phase stamps and a
bit-identity check against the first variant.

usage: python tools/diag/nt_bench.py [VARIANT ...]   VARIANT = "ENV=V,ENV=V" (empty: defaults)
"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import torch
from irlmx import DeviceMDP, ops
dev = torch.device("cuda", 0)
size, B = int(os.environ.get("SIZE", 128)), int(os.environ.get("B", 64))
n = size * size
mdp = DeviceMDP.icy_gridworld(size, np.linspace(0.1, 0.3, B), device=dev)
tm = ops.terminal_mask([n - 1], n, batch=B, device=dev)
r = torch.ones((B, n), dtype=torch.float64, device=dev)
variants = sys.argv[1:] or [""]
RESC = os.environ.get("RESCALE", "1") != "0"
keys = ("IRLMX_NT", "IRLMX_PAIR", "IRLMX_CLUSTER_R", "IRLMX_CLUSTER_G", "IRLMX_STAMPS", "IRLMX_BALANCED")
ref = None
for v in variants:
    for k in keys:
        os.environ.pop(k, None)
    for kv in filter(None, v.split(",")):
        k, val = kv.split("=")
        os.environ[k] = val
    pi = ops.backward_maxent(mdp, r, tm, rescale=RESC); torch.cuda.synchronize()
    ts = []
    for _ in range(4):
        t = time.perf_counter(); pi = ops.backward_maxent(mdp, r, tm, rescale=RESC); torch.cuda.synchronize(); ts.append(time.perf_counter() - t)
    same = None if ref is None else bool(torch.equal(ref, pi))
    if ref is None:
        ref = pi
    import hashlib
    h = hashlib.sha256(pi.cpu().numpy().tobytes()).hexdigest()[:16]
    print(f"[{v or 'default'}] backward {min(ts) * 1e3:.2f} ms  bit-identical to first: {same}  sha {h}", flush=True)
    os.environ["IRLMX_STAMPS"] = "1"
    ops.backward_maxent(mdp, r, tm, rescale=RESC); torch.cuda.synchronize()
    os.environ.pop("IRLMX_STAMPS")
