"""Cost of the drop-in backward (maxent.local_action_probabilities) in numpy's
order (one workgroup per instance, 2 S sweeps) against the tiled rescaled
shapes (IRLMX_NUMPY_ORDER=0), for grids 16x16 .. 64x64 (STENCIL5) and random
dense tables (DENSE layout).  usage: python tools/diag/np_bwd_cost.py"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd"), os.path.join(ROOT, "oracle")]
import torch
import maxent as M
import maxent_oracle as O
from irlmx import DeviceMDP, ops


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


cases = [(f"grid {n}x{n}", O.icy_gridworld_table(n, 0.2)) for n in (16, 24, 32, 33, 40, 48, 56, 64)]
rng = np.random.default_rng(0)
for S in (256, 1024, 2048):
    P = rng.random((S, S, 4)) + 1e-3
    P /= P.sum(axis=1, keepdims=True)
    cases.append((f"dense S={S}", P))
for name, P in cases:
    S = P.shape[0]
    mdp = DeviceMDP.resident(P)
    r = -np.log(4.0) + rng.uniform(-0.05, 0.05, S)
    os.environ.pop("IRLMX_NUMPY_ORDER", None)
    t_np = timed(lambda: M.local_action_probabilities(mdp, [S - 1], r))
    os.environ["IRLMX_NUMPY_ORDER"] = "0"
    t_tl = timed(lambda: M.local_action_probabilities(mdp, [S - 1], r))
    os.environ.pop("IRLMX_NUMPY_ORDER", None)
    phi = [S - 1]
    t_snp = timed(lambda: M.local_causal_action_probabilities(mdp, phi, r + 1.0, 0.7))
    os.environ["IRLMX_NUMPY_ORDER"] = "0"
    t_stl = timed(lambda: M.local_causal_action_probabilities(mdp, phi, r + 1.0, 0.7))
    os.environ.pop("IRLMX_NUMPY_ORDER", None)
    print(f"{name:14s} S={S:5d} layout={mdp.layout}: backward numpy order {t_np:8.2f} ms, tiled {t_tl:8.2f} ms "
          f"(x{t_np / t_tl:5.1f}); soft VI numpy order {t_snp:8.2f} ms, other {t_stl:8.2f} ms (x{t_snp / t_stl:5.1f})",
          flush=True)
