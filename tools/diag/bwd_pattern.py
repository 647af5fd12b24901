import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import torch
from irlmx import DeviceMDP, ops
def setenv(env):
    for k in ("IRLMX_FUSED_MAX_STATES", "IRLMX_CLUSTER", "IRLMX_CLUSTER_R", "IRLMX_CLUSTER_G"):
        os.environ.pop(k, None)
    os.environ.update(env)
dev = torch.device("cuda", 0)
for size in (3, 4, 8):
    n = size * size
    mdp = DeviceMDP.icy_gridworld(size, 0.2, device=dev)
    tm = ops.terminal_mask([n - 1], n, device=dev)
    for r in (np.ones(n), np.zeros(n)):
        setenv({}); a = ops.backward_maxent(mdp, r, tm, rescale=False)[0].cpu().numpy()
        setenv({"IRLMX_FUSED_MAX_STATES": "0", "IRLMX_CLUSTER_R": str(size), "IRLMX_CLUSTER_G": "1"})
        b = ops.backward_maxent(mdp, r, tm, rescale=False)[0].cpu().numpy()
        bad = sorted(set(int(s) for s, _ in np.argwhere(a != b)))
        print(size, r[0], [(s % size, s // size) for s in bad])
