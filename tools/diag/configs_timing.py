"""Wall time of the hot-path calls at the BASELINE configs other than the bench's
config 3 (config 2: 64x64 single instance; config 5: causal 128x128; config 4:
256x256, 32 instances per GPU), plus the plan each call takes."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import torch
from irlmx import DeviceMDP, ops
from irlmx.batch import terminal_reward
dev = torch.device("cuda", 0)


def timed(fn, reps=2):
    fn(); torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t = time.perf_counter(); out = fn(); torch.cuda.synchronize(); best = min(best, time.perf_counter() - t)
    return best, out


for name, size, B in (("config2", 64, 1), ("config5", 128, 1), ("config4", 256, 32)):
    n = size * size
    mdp = DeviceMDP.icy_gridworld(size, np.linspace(0.1, 0.3, B) if B > 1 else 0.2, device=dev)
    tm = ops.terminal_mask([n - 1], n, batch=B, device=dev)
    rng = np.random.default_rng(5)
    r = torch.as_tensor(rng.uniform(0, 1.5, (B, n)) if name == "config5" else np.ones((B, n)), device=dev)
    p0 = torch.zeros((B, n), dtype=torch.float64, device=dev); p0[:, 0] = 1.0
    if name == "config5":
        phi = terminal_reward([n - 1], n, B, dev)
        tb, (pi, v, k, st) = timed(lambda: ops.soft_backward(mdp, r, phi, 0.7))
        what = f"soft VI {int(k.max())} sweeps"
    else:
        tb, pi = timed(lambda: ops.backward_maxent(mdp, r, tm))
        what = f"backward {2 * n} sweeps"
    tf, (svf, kf, st) = timed(lambda: ops.forward_svf(mdp, p0, tm, pi), reps=1)
    print(f"{name}: {what} {tb * 1e3:.1f} ms; forward {int(kf.max())} sweeps {tf * 1e3:.1f} ms "
          f"({tf / max(int(kf.max()), 1) * 1e6:.2f} us/sweep)", flush=True)
