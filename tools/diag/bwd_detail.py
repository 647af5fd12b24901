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
for size in (2, 3):
    n = size * size
    mdp = DeviceMDP.icy_gridworld(size, 0.2, device=dev)
    tm = ops.terminal_mask([n - 1], n, device=dev)
    r = np.ones(n)
    setenv({})
    a = ops.backward_maxent(mdp, r, tm, rescale=False)[0].cpu().numpy()
    setenv({"IRLMX_FUSED_MAX_STATES": "0", "IRLMX_CLUSTER_R": str(size), "IRLMX_CLUSTER_G": "1"})
    b = ops.backward_maxent(mdp, r, tm, rescale=False)[0].cpu().numpy()
    # extended precision reference of the same recurrence
    P = O.icy_gridworld_table(size, 0.2).astype(np.longdouble)
    er = np.exp(np.longdouble(1.0)) * np.ones(n, dtype=np.longdouble)
    zs = np.zeros(n, dtype=np.longdouble); zs[n - 1] = 1
    for _ in range(2 * n):
        za = np.array([er * P[:, :, k].dot(zs) for k in range(4)]).T
        zs = za.sum(axis=1)
    ex = (za / zs[:, None])
    print(size, "diff entries", np.argwhere(a != b).tolist()[:10])
    print("  fused err", float(np.max(np.abs(a - ex))), "cluster err", float(np.max(np.abs(b - ex))))
    dev_exp = torch.exp(torch.tensor([1.0], dtype=torch.float64, device=dev)).item()
    print("  exp(1) device", repr(dev_exp), "numpy", repr(np.exp(1.0)))
    if size == 3 and os.path.exists(os.path.join(ROOT, "tools/diag/pi_emul.npy")):
        em = np.load(os.path.join(ROOT, "tools/diag/pi_emul.npy"))
        print("  fused == emulation:", np.array_equal(a, em), " cluster == emulation:", np.array_equal(b, em))
        print("  state2 fused", a[2].tolist(), "\n  state2 clust", b[2].tolist(), "\n  state2 emul ", em[2].tolist())
