"""One 128x128 instance's backward (the full run's tail: a single instance's
32,767-sweep chain) under forced cluster plans, the planner's choice first.
usage: python tools/diag/bwd_plans.py [size B]"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import torch
from irlmx import DeviceMDP, ops
dev = torch.device("cuda", 0)
size = int(sys.argv[1]) if len(sys.argv) > 1 else 128
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
n = size * size
mdp = DeviceMDP.icy_gridworld(size, np.linspace(0.1, 0.3, B), device=dev)
tm = ops.terminal_mask([n - 1], n, batch=B, device=dev)
r = torch.as_tensor(np.random.default_rng(5).uniform(0, 1.5, (B, n)), device=dev)
ref = None
for R, G in [(0, 0), (2, 14), (2, 16), (3, 14), (4, 10), (4, 14), (4, 16), (6, 12), (8, 8), (8, 12), (8, 16),
             (16, 8), (16, 16)]:
    for k in ("IRLMX_CLUSTER_R", "IRLMX_CLUSTER_G"):
        os.environ.pop(k, None)
    if R:
        os.environ["IRLMX_CLUSTER_R"], os.environ["IRLMX_CLUSTER_G"] = str(R), str(G)
    try:
        plan = ops.execution_plan(mdp, "backward")
        pi = ops.backward_maxent(mdp, r, tm)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(3):
            pi = ops.backward_maxent(mdp, r, tm)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / 3
    except Exception as e:
        print(f"R={R} G={G}: {e}", flush=True)
        continue
    same = ref is None or torch.equal(pi, ref)
    ref = pi if ref is None else ref
    print(f"R={plan['R']:3d} G={plan['G']:3d} C={plan['C']:3d} spt={plan['spt']:3d} layout={plan['layout']}: "
          f"{dt * 1e3:.3f} ms  bit-identical={same}", flush=True)
