"""Fixed vs per-sweep cost of the config-3 forward (128x128, B = 64): forward
calls capped at K sweeps for several K, on the unit-reward policy; a linear fit
of call time against K separates the per-call overhead from the sweep rate."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import torch  # noqa: E402
from irlmx import DeviceMDP, ops  # noqa: E402

dev = torch.device("cuda", 0)
size, B = int(os.environ.get("SIZE", 128)), int(os.environ.get("B", 64))
n = size * size
mdp = DeviceMDP.icy_gridworld(size, np.linspace(0.1, 0.3, B), device=dev)
tm = ops.terminal_mask([n - 1], n, batch=B, device=dev)
r = torch.ones((B, n), dtype=torch.float64, device=dev)
p0 = torch.zeros((B, n), dtype=torch.float64, device=dev); p0[:, 0] = 1.0
pi = ops.backward_maxent(mdp, r, tm)
print("plan", ops.execution_plan(mdp, "forward"), flush=True)
ks, ts = [], []
for K in (8, 16, 64, 256, 1024, 4096):
    ops.forward_svf(mdp, p0, tm, pi, max_iter=K); torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        t = time.perf_counter(); ops.forward_svf(mdp, p0, tm, pi, max_iter=K); torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    ks.append(K); ts.append(best * 1e3)
    print(f"K={K:5d}  {best * 1e3:.3f} ms", flush=True)
slope, icpt = np.polyfit(ks, ts, 1)
print(f"fit: {icpt:.3f} ms per call + {slope * 1e3:.3f} us per sweep", flush=True)
if os.environ.get("STAMPS"):
    os.environ["IRLMX_STAMPS"] = "1"
    ops.forward_svf(mdp, p0, tm, pi, max_iter=16); torch.cuda.synchronize()
