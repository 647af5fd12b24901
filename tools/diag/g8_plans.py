"""The planner's backward plan against the best plan with G = 8 ghost rows
(IRLMX_CLUSTER_G=8) for 128x128 working sets of 1..64 instances (the full
run's compaction sizes).  usage: python tools/diag/g8_plans.py"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import torch
from irlmx import DeviceMDP, ops
from irlmx.shard import instance_slips
dev = torch.device("cuda", 0)
n = 128 * 128
for B in (1, 4, 8, 12, 16, 20, 24, 28, 32, 36, 40, 48, 56, 64):
    mdp = DeviceMDP.icy_gridworld(128, instance_slips(np.arange(B), 64), device=dev)
    tm = ops.terminal_mask([n - 1], n, batch=B, device=dev)
    r = torch.ones((B, n), dtype=torch.float64, device=dev)
    out, ref = [], None
    for G in (0, 8):
        os.environ.pop("IRLMX_CLUSTER_G", None)
        if G:
            os.environ["IRLMX_CLUSTER_G"] = str(G)
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
        out.append(f"{'planner' if not G else 'G=8'} ({plan['R']},{plan['G']},{plan['C']}) spt {plan['spt']}: "
                   f"{np.median(ts):.2f} ms{'' if same else ' DIFFERS'}")
    os.environ.pop("IRLMX_CLUSTER_G", None)
    print(f"B={B:2d}: " + " | ".join(out), flush=True)
