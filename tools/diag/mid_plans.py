"""Backward wall time of 128x128 batches between 9 and 48 instances (the full
run's compacted working sets) under forced cluster plans (IRLMX_CLUSTER_R / _G),
the planner's choice first: which plans the cost model misjudges.
usage: python tools/diag/mid_plans.py"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import torch
from irlmx import DeviceMDP, ops
from irlmx.shard import instance_slips
dev = torch.device("cuda", 0)
n = 128 * 128
CASES = {12: [(0, 0), (8, 12), (8, 8), (10, 10), (12, 10), (16, 8)],
         20: [(0, 0), (14, 9), (16, 8), (12, 10), (14, 8), (10, 10), (8, 12)],
         36: [(0, 0), (22, 9), (22, 8), (24, 8), (20, 10), (26, 11), (26, 10), (32, 8)],
         44: [(0, 0), (26, 11), (26, 10), (28, 10), (32, 8)]}
for B, plans in CASES.items():
    mdp = DeviceMDP.icy_gridworld(128, instance_slips(np.arange(B), 64), device=dev)
    tm = ops.terminal_mask([n - 1], n, batch=B, device=dev)
    r = torch.ones((B, n), dtype=torch.float64, device=dev)
    ref = None
    for R, G in plans:
        for k in ("IRLMX_CLUSTER_R", "IRLMX_CLUSTER_G"):
            os.environ.pop(k, None)
        if R:
            os.environ["IRLMX_CLUSTER_R"], os.environ["IRLMX_CLUSTER_G"] = str(R), str(G)
        plan = ops.execution_plan(mdp, "backward")
        pi = ops.backward_maxent(mdp, r, tm)
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            t = time.perf_counter()
            ops.backward_maxent(mdp, r, tm)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t) * 1e3)
        same = ref is None or torch.equal(pi, ref)
        ref = pi if ref is None else ref
        print(f"B={B:2d} {'planner' if not R else 'forced '} R={plan['R']:2d} G={plan['G']:2d} C={plan['C']:2d} "
              f"spt={plan['spt']:2d} launches={plan['launches']}: {np.median(ts):7.3f} ms  bit-identical={same}",
              flush=True)
    for k in ("IRLMX_CLUSTER_R", "IRLMX_CLUSTER_G"):
        os.environ.pop(k, None)
