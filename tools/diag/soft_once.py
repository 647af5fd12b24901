"""One config-5 soft VI call (128x128, fp64, discount 0.7), for kernel traces."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import torch
from irlmx import DeviceMDP, ops
from irlmx.batch import terminal_reward
dev = torch.device("cuda", 0)
size = int(os.environ.get("SIZE", 128)); n = size * size
mdp = DeviceMDP.icy_gridworld(size, 0.2, device=dev)
r = torch.as_tensor(np.random.default_rng(5).uniform(0, 1.5, (1, n)), device=dev)
phi = terminal_reward([n - 1], n, 1, dev)
for _ in range(2):
    torch.cuda.synchronize(); t = time.perf_counter()
    pi, v, k, st = ops.soft_backward(mdp, r, phi, 0.7)
    torch.cuda.synchronize()
    print(f"soft VI {int(k[0])} sweeps {1e3 * (time.perf_counter() - t):.2f} ms", flush=True)

v, kv, _ = ops.value_iteration(mdp, r, 0.9)
torch.cuda.synchronize(); t = time.perf_counter()
v, kv, _ = ops.value_iteration(mdp, r, 0.9)
torch.cuda.synchronize()
print(f"VI {int(kv[0])} sweeps {1e3 * (time.perf_counter() - t):.2f} ms", flush=True)
