import os, sys, time
import numpy as np
sys.path[:0] = ["/root/repo/irl-maxent_amd"]
import torch
from irlmx import DeviceMDP, ops
from irlmx.batch import terminal_reward
dev = torch.device("cuda", 0)
n = 128 * 128
mdp = DeviceMDP.icy_gridworld(128, 0.2, device=dev)
tm = ops.terminal_mask([n - 1], n, device=dev)
r = torch.as_tensor(np.random.default_rng(5).uniform(0, 1.5, (1, n)), device=dev)
phi = terminal_reward([n - 1], n, 1, dev)
pi, v, k, st = ops.soft_backward(mdp, r, phi, 0.7)
print("soft", int(k[0]), flush=True)
p0 = torch.zeros((1, n), dtype=torch.float64, device=dev); p0[:, 0] = 1.0
os.environ["IRLMX_STAMPS"] = "1"
t = time.perf_counter(); svf, kf, st = ops.forward_svf(mdp, p0, tm, pi); torch.cuda.synchronize()
print("fwd", int(kf[0]), int(st[0]), time.perf_counter() - t, flush=True)
