"""Generic-sparsity (ELL) loops on the grid shape vs the per-sweep shape:
microseconds per sweep of backward, capped forward, soft VI, VI.  Default: the
128x128 IcyGridWorld in ELL form (5 slots); `wide`: the 6000-state random sparse
models of test_ell_grid_shape_wide_rows (12 and 24 successors per state)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np, torch
import maxent_oracle as O
from irlmx import ops
from irlmx.batch import terminal_reward
from test_gpu_full_size import ell_model, random_sparse_mats

dev = torch.device("cuda", 0)
if "wide" in sys.argv[1:]:
    models = [(f"random sparse S=6000, {k} successors", ell_model(random_sparse_mats(6000, 4, k, seed=k), dev))
              for k in (12, 24)]
else:
    models = [("IcyGridWorld 128x128 in ELL", ell_model(O.icy_gridworld_csr(128, 0.2), dev))]
for label, mdp in models:
  n = mdp.n_states
  print(f"== {label}: k_row {mdp.k_row}, k_col {mdp.k_col}", flush=True)
  r = np.random.default_rng(1).uniform(0, 1, (1, n))
  tm = ops.terminal_mask([n - 1], n, device=dev)
  p0 = np.zeros((1, n)); p0[0, 0] = 1.0
  phi = terminal_reward([n - 1], n, 1, dev)
  pi = ops.backward_maxent(mdp, r, tm)
  for grid in ("1", "0"):
      os.environ["IRLMX_GRID"] = grid
      for name, fn, sweeps in (("backward", lambda: ops.backward_maxent(mdp, r, tm), 2 * n),
                               ("forward (<= 3000 sweeps)", lambda: ops.forward_svf(mdp, p0, tm, pi, max_iter=3000), None),
                               ("soft VI", lambda: ops.soft_backward(mdp, r, phi, 0.7), None),
                               ("VI", lambda: ops.value_iteration(mdp, r, 0.9), None)):
          out = fn(); torch.cuda.synchronize()
          t = time.perf_counter(); out = fn(); torch.cuda.synchronize(); dt = time.perf_counter() - t
          k = sweeps or int(out[2][0] if name == "soft VI" else out[1][0])
          print(f"{'grid ' if grid == '1' else 'sweep'} {name}: {k} sweeps {dt * 1e3:.1f} ms = {dt / k * 1e6:.2f} us/sweep",
                flush=True)
