"""Is power-of-two rescaling exact in each shape?  Compare rescale on/off at r = 0 and r = 1."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd"), os.path.join(ROOT, "oracle")]
import torch
from irlmx import DeviceMDP, ops
import maxent_oracle as O

def setenv(env):
    for k in ("IRLMX_FUSED_MAX_STATES", "IRLMX_CLUSTER", "IRLMX_CLUSTER_R", "IRLMX_CLUSTER_G"):
        os.environ.pop(k, None)
    os.environ.update(env)

dev = torch.device("cuda", 0)
size, n = 8, 64
mdp = DeviceMDP.icy_gridworld(size, 0.2, device=dev)
tm = ops.terminal_mask([n - 1], n, device=dev)
P = O.icy_gridworld_table(size, 0.2)
for rv in (0.0, 1.0):
    r = np.full(n, rv)
    ref = O.backward_maxent(P, [n - 1], r)
    for name, env in (("fused", {}), ("sweep", {"IRLMX_FUSED_MAX_STATES": "0", "IRLMX_CLUSTER": "0"}),
                      ("cluster", {"IRLMX_FUSED_MAX_STATES": "0", "IRLMX_CLUSTER_R": "8", "IRLMX_CLUSTER_G": "1"})):
        setenv(env)
        on = ops.backward_maxent(mdp, r, tm, rescale=True)[0].cpu().numpy()
        off = ops.backward_maxent(mdp, r, tm, rescale=False)[0].cpu().numpy()
        print(f"r={rv} {name:7s}: on==off {np.array_equal(on, off)} max {np.max(np.abs(on - off)):.2e}; "
              f"on vs oracle {np.max(np.abs(on - ref)):.2e}; off vs oracle {np.max(np.abs(off - ref)):.2e}")
