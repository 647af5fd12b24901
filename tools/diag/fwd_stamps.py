"""Phase stamps (IRLMX_STAMPS=1) of the forward at config 3's plan (128x128,
B = 64, a capped 3,000-sweep call) and of one 128x128 instance (config 5's
shape, 20,000 sweeps): cycles per block in sweeps / publish / wait / refresh.
usage: python tools/diag/fwd_stamps.py"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import torch
from irlmx import DeviceMDP, ops
from irlmx.shard import instance_slips
dev = torch.device("cuda", 0)
for B, cap in ((64, 3000), (1, 20000)):
    n = 128 * 128
    mdp = DeviceMDP.icy_gridworld(128, instance_slips(np.arange(B), B), device=dev)
    tm = ops.terminal_mask([n - 1], n, batch=B, device=dev)
    r = torch.ones((B, n), dtype=torch.float64, device=dev)
    pi = ops.backward_maxent(mdp, r, tm)
    p0 = torch.zeros((B, n), dtype=torch.float64, device=dev)
    p0[:, 0] = 1.0
    ops.forward_svf(mdp, p0, tm, pi, max_iter=cap)
    torch.cuda.synchronize()
    os.environ["IRLMX_STAMPS"] = "1"
    print(f"B={B} cap={cap}", ops.execution_plan(mdp, "forward"), flush=True)
    ops.forward_svf(mdp, p0, tm, pi, max_iter=cap)
    torch.cuda.synchronize()
    os.environ.pop("IRLMX_STAMPS")
