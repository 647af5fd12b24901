"""Separate backward and forward bitwise comparisons across shapes (same inputs)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd"), os.path.join(ROOT, "oracle")]
import torch
from irlmx import DeviceMDP, ops

def setenv(env):
    for k in ("IRLMX_FUSED_MAX_STATES", "IRLMX_CLUSTER", "IRLMX_CLUSTER_R", "IRLMX_CLUSTER_G"):
        os.environ.pop(k, None)
    os.environ.update(env)

dev = torch.device("cuda", 0)
size, n = 8, 64
r = np.ones(n)
p0 = np.zeros(n); p0[0] = 1.0
mdp = DeviceMDP.icy_gridworld(size, 0.2, device=dev)
tm = ops.terminal_mask([n - 1], n, device=dev)
setenv({})
pi_f = ops.backward_maxent(mdp, r, tm)
svf_f, kf, _ = ops.forward_svf(mdp, p0, tm, pi_f)
for R, G in ((8, 1), (3, 2), (4, 1), (2, 2)):
    setenv({"IRLMX_FUSED_MAX_STATES": "0", "IRLMX_CLUSTER_R": str(R), "IRLMX_CLUSTER_G": str(G)})
    pi_c = ops.backward_maxent(mdp, r, tm)
    svf_c, kc, _ = ops.forward_svf(mdp, p0, tm, pi_f)   # same policy as the fused run
    d = (pi_f - pi_c).abs()
    print(f"R={R} G={G}: backward bitwise={bool(torch.equal(pi_f, pi_c))} max={d.max().item():.3e} "
          f"n_diff={(d > 0).sum().item()}; forward(same pi) bitwise={bool(torch.equal(svf_f, svf_c))} "
          f"max={(svf_f - svf_c).abs().max().item():.3e} k={int(kf[0])}/{int(kc[0])}")
# rescale off: compare raw (no power-of-two shifts) -- S=64 gives 127 sweeps, no overflow at r=1? growth ~10/sweep
setenv({})
pi_f0 = ops.backward_maxent(mdp, np.zeros(n), tm, rescale=False)
setenv({"IRLMX_FUSED_MAX_STATES": "0", "IRLMX_CLUSTER_R": "8", "IRLMX_CLUSTER_G": "1"})
pi_c0 = ops.backward_maxent(mdp, np.zeros(n), tm, rescale=False)
print("no-rescale r=0 single tile bitwise:", bool(torch.equal(pi_f0, pi_c0)), (pi_f0 - pi_c0).abs().max().item())
