import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import torch
from irlmx import DeviceMDP, ops
dev = torch.device("cuda", 0)
size, B = 128, 64
n = size * size
mdp = DeviceMDP.icy_gridworld(size, np.linspace(0.1, 0.3, B), device=dev)
tm = ops.terminal_mask([n - 1], n, batch=B, device=dev)
r = torch.ones((B, n), dtype=torch.float64, device=dev)
os.environ.pop("IRLMX_STRIP", None)
ref = ops.backward_maxent(mdp, r, tm); torch.cuda.synchronize()
os.environ["IRLMX_STAMPS"] = "1"
for strip in ("0", "1"):
    os.environ["IRLMX_STRIP"] = strip
    t = time.perf_counter(); out = ops.backward_maxent(mdp, r, tm); torch.cuda.synchronize(); dt = time.perf_counter() - t
    print(f"strip={strip}: {dt*1e3:.2f} ms  bitwise={bool(torch.equal(out, ref))}", flush=True)
