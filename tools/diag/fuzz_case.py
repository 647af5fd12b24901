"""Run one tests/test_gpu_plan_fuzz.py case phase by phase with timings
(python tools/diag/fuzz_case.py INDEX [CAP]): cluster then per-sweep shape,
backward and forward separately."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "irl-maxent_amd")]
import torch  # noqa: E402,F401
import test_gpu_plan_fuzz as F  # noqa: E402
from conftest import icy_stencil_rect  # noqa: E402
from irlmx import DeviceMDP, _lib, ops, require_device  # noqa: E402

idx = int(sys.argv[1])
cap_override = int(sys.argv[2]) if len(sys.argv) > 2 else None
rng = np.random.default_rng(20261018)
for i in range(idx + 1):
    c = F.draw(rng)
if cap_override is not None:
    c["cap"] = cap_override
print(c, flush=True)
dev = require_device()
W, H, B = c["W"], c["H"], c["B"]
S = W * H
r_ = np.random.default_rng(c["seed"])
slips = r_.uniform(0.05, 0.4, B)
if W == H and r_.random() < 0.5:
    mdp = DeviceMDP.icy_gridworld(W, slips, device=dev)
else:
    rv = np.stack([icy_stencil_rect(W, H, p) for p in slips])
    mdp = DeviceMDP(_lib.LAYOUT_STENCIL5, S, 4, B, False, torch.as_tensor(rv, device=dev), width=W, height=H,
                    device=dev)
reward = r_.uniform(-1.0 if c["neg"] else 0.0, 1.5, (B, S))
terminal = sorted(set([S - 1] + [int(t) for t in r_.integers(0, S, int(r_.integers(0, 3)))]))
tm = ops.terminal_mask(terminal, S, batch=B, device=dev)
p0 = r_.random((B, S)) ** 8
p0 /= p0.sum(axis=1, keepdims=True)
env = {"IRLMX_FUSED_MAX_STATES": 0, "IRLMX_CLUSTER_R": c["R"], "IRLMX_CLUSTER_G": c["G"]}
if c["layout"] >= 0:
    env["IRLMX_PAIR"] = c["layout"]
for name, e in (("cluster", env), ("sweep", {"IRLMX_FUSED_MAX_STATES": 0, "IRLMX_CLUSTER": 0})):
    for k in F.KEYS:
        os.environ.pop(k, None)
    os.environ.update({k: str(v) for k, v in e.items()})
    print(name, [ops.execution_plan(mdp, op) for op in ("backward", "forward")], flush=True)
    t = time.time()
    pi = ops.backward_maxent(mdp, reward, tm)
    torch.cuda.synchronize()
    print(f"  backward {time.time() - t:.3f}s finite={bool(torch.isfinite(pi).all())}", flush=True)
    t = time.time()
    svf, k, st = ops.forward_svf(mdp, p0, tm, pi, max_iter=c["cap"])
    torch.cuda.synchronize()
    print(f"  forward {time.time() - t:.3f}s k={k.tolist()} status={st.tolist()}", flush=True)
