"""Time the cluster backward at 128x128 x 64 for several (R, G) plans to split sweep vs exchange cost."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import torch
from irlmx import DeviceMDP, ops
dev = torch.device("cuda", 0)
size, B = int(os.environ.get("SIZE", "128")), int(os.environ.get("B", "64"))
n = size * size
mdp = DeviceMDP.icy_gridworld(size, np.linspace(0.1, 0.3, B), device=dev)
tm = ops.terminal_mask([n - 1], n, batch=B, device=dev)
r = torch.ones((B, n), dtype=torch.float64, device=dev)
for R, G in ((32, 8), (32, 4), (32, 2), (32, 1), (40, 4), (16, 16), (24, 12)):
    os.environ["IRLMX_CLUSTER_R"] = str(R); os.environ["IRLMX_CLUSTER_G"] = str(G)
    try:
        ops.backward_maxent(mdp, r, tm); torch.cuda.synchronize()
        t = time.perf_counter(); ops.backward_maxent(mdp, r, tm); torch.cuda.synchronize(); dt = time.perf_counter() - t
        blocks = (2 * n - 1 + G - 1) // G
        print(f"R={R:3d} G={G:2d}: {dt*1e3:8.2f} ms  {dt/(2*n)*1e6:6.2f} us/sweep  {dt/blocks*1e6:7.2f} us/block", flush=True)
    except Exception as e:
        print(R, G, "error", e)
