"""Persistent dense shape vs per-sweep dense kernels: microseconds per sweep of
the collapsed backward (2S - 1 sweeps + the per-action sweep) and the forward,
on random dense tables (shared for B > 1), for the planner's rows per workgroup
and every other RB that fits.  usage: python tools/diag/dense_grid_bench.py [S ...]
(BATCHES=1,2 by default; RBS=4,8,16 to restrict the forced variants)"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import numpy as np, torch
from irlmx import DeviceMDP, ops
from irlmx.batch import terminal_reward

dev = torch.device("cuda", 0)


def timed(fn, reps=3):
    fn(); torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        t = time.perf_counter(); out = fn(); torch.cuda.synchronize(); best = min(best, time.perf_counter() - t)
    return best, out


sizes = [int(a) for a in sys.argv[1:]] or [512, 1024, 2048, 4096]
for S in sizes:
    rng = np.random.default_rng(S)
    P = rng.random((S, S, 4)) + 1e-3
    P /= P.sum(axis=1, keepdims=True)
    one = DeviceMDP.from_dense(P, device=dev, layout="dense")
    del P
    for B in [int(x) for x in os.environ.get("BATCHES", "1,2").split(",")]:
        mdp = one.with_batch(B)
        r = rng.uniform(0.0, 1.0, (B, S))
        tm = ops.terminal_mask([S - 1], S, batch=B, device=dev)
        p0 = np.zeros((B, S)); p0[:, 0] = 1.0
        pi = ops.backward_maxent(mdp, r, tm)
        variants = [("per-sweep", {"IRLMX_DENSE_GRID": "0"}), ("planner", {})]
        for rb in [int(x) for x in os.environ.get("RBS", "4,8,16,32,64").split(",")]:
            variants.append((f"rb={rb}", {"IRLMX_DENSE_GRID_RB": str(rb), "IRLMX_DENSE_GRID_XCD": "0"}))
            variants.append((f"rb={rb} xcd", {"IRLMX_DENSE_GRID_RB": str(rb), "IRLMX_DENSE_GRID_XCD": "1"}))
        for name, env in variants:
            for k in ("IRLMX_DENSE_GRID", "IRLMX_DENSE_GRID_RB", "IRLMX_DENSE_GRID_XCD"):
                os.environ.pop(k, None)
            os.environ.update(env)
            plan = ops.execution_plan(mdp, "backward")
            if name.startswith("rb=") and (plan["shape"] != "dense-grid" or plan["R"] != int(name.split()[0][3:])):
                continue
            tb, _ = timed(lambda: ops.backward_maxent(mdp, r, tm))
            tf, (svf, k, _) = timed(lambda: ops.forward_svf(mdp, p0, tm, pi, max_iter=4000))
            kk = int(k.max())
            phi = terminal_reward([S - 1], S, B, dev)
            ps = ops.execution_plan(mdp, "soft_backward")
            tsv, (_, _, ks, _) = timed(lambda: ops.soft_backward(mdp, r, phi, 0.7))
            tvi, (_, kv, _) = timed(lambda: ops.value_iteration(mdp, r, 0.9))
            print(f"S={S} B={B} {name:13s} [{plan['shape']} R={plan['R']} C={plan['C']} cpt={plan['spt']} xcd={plan['G']}]: "
                  f"backward {tb * 1e3:.2f} ms = {tb / (2 * S) * 1e6:.2f} us/sweep; forward {kk} sweeps "
                  f"{tf * 1e3:.2f} ms = {tf / kk * 1e6:.2f} us/sweep; [{ps['shape']} R={ps['R']} xcd={ps['G']}] "
                  f"soft VI {int(ks.max())} sweeps {tsv / int(ks.max()) * 1e6:.2f} us/sweep; "
                  f"VI {int(kv.max())} sweeps {tvi / int(kv.max()) * 1e6:.2f} us/sweep", flush=True)
        for k in ("IRLMX_DENSE_GRID", "IRLMX_DENSE_GRID_RB", "IRLMX_DENSE_GRID_XCD"):
            os.environ.pop(k, None)
