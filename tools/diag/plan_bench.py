"""Forward / backward wall time under forced cluster plans (env overrides), with
a bit-identity check against the first variant and phase stamps.

usage: SIZE=64 B=1 MODE=fwd python tools/diag/plan_bench.py [VARIANT ...]
       VARIANT = "ENV=V,ENV=V" (empty string: the default plan)
"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import torch
from irlmx import DeviceMDP, ops
dev = torch.device("cuda", 0)
size, B, mode = int(os.environ.get("SIZE", 64)), int(os.environ.get("B", 1)), os.environ.get("MODE", "fwd")
n = size * size
mdp = DeviceMDP.icy_gridworld(size, np.linspace(0.1, 0.3, B) if B > 1 else 0.2, device=dev)
tm = ops.terminal_mask([n - 1], n, batch=B, device=dev)
rng = np.random.default_rng(5)
r = torch.as_tensor(rng.uniform(0, 1.5, (B, n)) if os.environ.get("RAND") else np.ones((B, n)), device=dev)
p0 = torch.zeros((B, n), dtype=torch.float64, device=dev); p0[:, 0] = 1.0
keys = ("IRLMX_NT", "IRLMX_PAIR", "IRLMX_CLUSTER_R", "IRLMX_CLUSTER_G", "IRLMX_STAMPS", "IRLMX_CLUSTER", "IRLMX_FUSED",
        "IRLMX_DEFER", "IRLMX_FWD_LAG", "IRLMX_EAGER_SUMMARY")
pi = ops.backward_maxent(mdp, r, tm)
torch.cuda.synchronize()
ref = None
for v in sys.argv[1:] or [""]:
    for k in keys:
        os.environ.pop(k, None)
    for kv in filter(None, v.split(",")):
        k, val = kv.split("=")
        os.environ[k] = val
    if mode == "fwd":
        call = lambda: ops.forward_svf(mdp, p0, tm, pi, max_iter=int(os.environ.get("MAXITER", "0")))[0:2]
    else:
        call = lambda: (ops.backward_maxent(mdp, r, tm), torch.zeros(1))
    out = call(); torch.cuda.synchronize()
    ts = []
    for _ in range(2):
        t = time.perf_counter(); out = call(); torch.cuda.synchronize(); ts.append(time.perf_counter() - t)
    same = None if ref is None else (bool(torch.equal(ref[0], out[0])) and bool(torch.equal(ref[1], out[1])))
    if ref is None:
        ref = out
    sweeps = int(out[1].max()) if mode == "fwd" else 2 * n
    pl = ops.execution_plan(mdp, "forward" if mode == "fwd" else "backward")
    print(f"[{v or 'default'}] {mode} {min(ts) * 1e3:.2f} ms  sweeps {sweeps}  {min(ts) / sweeps * 1e6:.3f} us/sweep  "
          f"identical: {same}  plan {pl['shape']} R={pl['R']} G={pl['G']} C={pl['C']} spt={pl['spt']}", flush=True)
    if os.environ.get("STAMPS"):
        os.environ["IRLMX_STAMPS"] = "1"
        call(); torch.cuda.synchronize()
        os.environ.pop("IRLMX_STAMPS")
