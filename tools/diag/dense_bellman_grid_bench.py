"""Dense soft VI / VI on the persistent dense shape: microseconds per sweep for
every rows-per-workgroup choice, spread over the chip and XCD-grouped, against
the per-sweep dense kernels.  usage: python tools/diag/dense_bellman_grid_bench.py [S ...]"""
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


for S in [int(a) for a in sys.argv[1:]] or [256, 512, 1024]:
    rng = np.random.default_rng(S)
    P = rng.random((S, S, 4)) + 1e-3
    P /= P.sum(axis=1, keepdims=True)
    mdp = DeviceMDP.from_dense(P, device=dev, layout="dense")
    r = rng.uniform(0.0, 1.0, (1, S))
    phi = terminal_reward([S - 1], S, 1, dev)
    variants = [("per-sweep", {"IRLMX_DENSE_GRID": "0"}), ("planner", {})]
    for rb in (2, 4, 8, 16):
        for x in ("0", "1"):
            variants.append((f"rb={rb} xcd={x}", {"IRLMX_DENSE_GRID_RB": str(rb), "IRLMX_DENSE_GRID_XCD": x}))
    for name, env in variants:
        for k in ("IRLMX_DENSE_GRID", "IRLMX_DENSE_GRID_RB", "IRLMX_DENSE_GRID_XCD"):
            os.environ.pop(k, None)
        os.environ.update(env)
        p = ops.execution_plan(mdp, "soft_backward")
        if name.startswith("rb=") and (p["shape"] != "dense-grid" or p["R"] != int(name[3:].split()[0])
                                       or p["G"] != int(name[-1])):
            continue
        tsv, (_, _, ks, _) = timed(lambda: ops.soft_backward(mdp, r, phi, 0.7))
        tvi, (_, kv, _) = timed(lambda: ops.value_iteration(mdp, r, 0.9))
        print(f"S={S} {name:14s} [{p['shape']} R={p['R']} C={p['C']} xcd={p['G']}]: soft VI {int(ks[0])} sweeps "
              f"{tsv / int(ks[0]) * 1e6:.2f} us/sweep; VI {int(kv[0])} sweeps {tvi / int(kv[0]) * 1e6:.2f} us/sweep",
              flush=True)
