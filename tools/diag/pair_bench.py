"""Backward / forward cluster-kernel timing at config 3 (128x128, 64 instances):
per-state LDS layout (IRLMX_PAIR=0) vs the pair layout, with phase stamps."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import torch
from irlmx import DeviceMDP, ops
dev = torch.device("cuda", 0)
size, B = int(os.environ.get("SIZE", 128)), int(os.environ.get("B", 64))
n = size * size
mdp = DeviceMDP.icy_gridworld(size, np.linspace(0.1, 0.3, B), device=dev)
tm = ops.terminal_mask([n - 1], n, batch=B, device=dev)
r = torch.ones((B, n), dtype=torch.float64, device=dev)  # the reference's initial theta (Constant(1.0))
p0 = torch.zeros((B, n), dtype=torch.float64, device=dev); p0[:, 0] = 1.0
res = {}
for pair, xg in (("0", "1"), ("1", "1"), ("2", "1"), ("3", "1")):
    os.environ["IRLMX_PAIR"] = pair
    os.environ["IRLMX_XCD_GROUP"] = xg
    os.environ.pop("IRLMX_STAMPS", None)
    pi = ops.backward_maxent(mdp, r, tm); torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        t = time.perf_counter(); pi = ops.backward_maxent(mdp, r, tm); torch.cuda.synchronize(); ts.append(time.perf_counter() - t)
    svf, k, _ = ops.forward_svf(mdp, p0, tm, pi, max_iter=400000); torch.cuda.synchronize()
    tf = []
    for _ in range(3):
        t = time.perf_counter(); svf, k, _ = ops.forward_svf(mdp, p0, tm, pi, max_iter=400000); torch.cuda.synchronize(); tf.append(time.perf_counter() - t)
    res[pair + xg] = (pi, svf, k)
    print(f"pair={pair} xcd_group={xg}: backward {min(ts)*1e3:.2f} ms, forward {min(tf)*1e3:.2f} ms "
          f"(sweeps {int(k.max())})", flush=True)
    os.environ["IRLMX_STAMPS"] = "1"
    ops.backward_maxent(mdp, r, tm); torch.cuda.synchronize()
    os.environ.pop("IRLMX_STAMPS")
for k in ("11", "21", "31"):
    print("bit-identical", k, torch.equal(res["01"][0], res[k][0]), torch.equal(res["01"][1], res[k][1]),
          torch.equal(res["01"][2], res[k][2]))
