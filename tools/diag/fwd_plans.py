"""One 128x128 instance's forward (config 5's shape: the causal forward runs
~170,000 sweeps per step) under forced cluster plans: microseconds per sweep of
a capped 20,000-sweep call, the planner's choice first.
usage: python tools/diag/fwd_plans.py [size]"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import torch
from irlmx import DeviceMDP, ops
dev = torch.device("cuda", 0)
size = int(sys.argv[1]) if len(sys.argv) > 1 else 128
n = size * size
mdp = DeviceMDP.icy_gridworld(size, 0.2, device=dev)
tm = ops.terminal_mask([n - 1], n, device=dev)
r = torch.as_tensor(np.random.default_rng(5).uniform(0, 1.5, (1, n)), device=dev)
pi = ops.backward_maxent(mdp, r, tm)
p0 = torch.zeros((1, n), dtype=torch.float64, device=dev)
p0[0, 0] = 1.0
cap = 20000
ref = None
for R, G in [(0, 0), (8, 8), (8, 12), (8, 16), (12, 8), (12, 12), (16, 8), (16, 12), (16, 16), (24, 8), (32, 8),
             (4, 10), (6, 8), (6, 12)]:
    for k in ("IRLMX_CLUSTER_R", "IRLMX_CLUSTER_G"):
        os.environ.pop(k, None)
    if R:
        os.environ["IRLMX_CLUSTER_R"], os.environ["IRLMX_CLUSTER_G"] = str(R), str(G)
    try:
        plan = ops.execution_plan(mdp, "forward")
        svf, k, st = ops.forward_svf(mdp, p0, tm, pi, max_iter=cap)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(3):
            svf, k, st = ops.forward_svf(mdp, p0, tm, pi, max_iter=cap)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / 3
    except Exception as e:   # a forced plan that does not fit
        print(f"R={R} G={G}: {e}", flush=True)
        continue
    same = ref is None or torch.equal(svf, ref)
    ref = svf if ref is None else ref
    print(f"R={plan['R']:3d} G={plan['G']:3d} C={plan['C']:3d} spt={plan['spt']:3d} layout={plan['layout']}: "
          f"{dt / cap * 1e6:.3f} us/sweep  bit-identical={same}", flush=True)
