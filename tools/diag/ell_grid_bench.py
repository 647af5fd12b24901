"""Generic-sparsity (ELL) loops at 128x128 on the grid shape vs the per-sweep
shape: microseconds per sweep of backward, capped forward, soft VI, VI."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np, torch
import maxent_oracle as O
from irlmx import ops
from irlmx.batch import terminal_reward
from test_gpu_full_size import ell_model

dev = torch.device("cuda", 0)
n = 128 * 128
mdp = ell_model(O.icy_gridworld_csr(128, 0.2), dev)
r = np.random.default_rng(1).uniform(0, 1, (1, n))
tm = ops.terminal_mask([n - 1], n, device=dev)
p0 = np.zeros((1, n)); p0[0, 0] = 1.0
phi = terminal_reward([n - 1], n, 1, dev)
pi = ops.backward_maxent(mdp, r, tm)
for grid in ("1", "0"):
    os.environ["IRLMX_GRID"] = grid
    for name, fn, sweeps in (("backward", lambda: ops.backward_maxent(mdp, r, tm), 2 * n),
                             ("forward (3000 sweeps)", lambda: ops.forward_svf(mdp, p0, tm, pi, max_iter=3000), 3000),
                             ("soft VI", lambda: ops.soft_backward(mdp, r, phi, 0.7), None),
                             ("VI", lambda: ops.value_iteration(mdp, r, 0.9), None)):
        out = fn(); torch.cuda.synchronize()
        t = time.perf_counter(); out = fn(); torch.cuda.synchronize(); dt = time.perf_counter() - t
        k = sweeps or int(out[2][0] if name == "soft VI" else out[1][0])
        print(f"{'grid ' if grid == '1' else 'sweep'} {name}: {k} sweeps {dt * 1e3:.1f} ms = {dt / k * 1e6:.2f} us/sweep",
              flush=True)
