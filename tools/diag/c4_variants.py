"""Config 4's backward (256x256, 32 instances) under forced plans and layouts,
with in-kernel phase stamps (IRLMX_STAMPS=1): wall time per call and cycles
per block by phase.  usage: python tools/diag/c4_variants.py [size B]"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import torch
from irlmx import DeviceMDP, ops
from irlmx.shard import instance_slips
dev = torch.device("cuda", 0)
size = int(sys.argv[1]) if len(sys.argv) > 1 else 256
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
n = size * size
mdp = DeviceMDP.icy_gridworld(size, instance_slips(np.arange(B), B), device=dev)
tm = ops.terminal_mask([n - 1], n, batch=B, device=dev)
r = torch.ones((B, n), dtype=torch.float64, device=dev)
variants = [("cw-default", {}), ("cw-R16G8", {"IRLMX_CLUSTER_R": "16", "IRLMX_CLUSTER_G": "8"}),
            ("cw-R24G8", {"IRLMX_CLUSTER_R": "24", "IRLMX_CLUSTER_G": "8"}),
            ("old", {"IRLMX_COMPACT": "0"})]
keys = ("IRLMX_CLUSTER_R", "IRLMX_CLUSTER_G", "IRLMX_COMPACT", "IRLMX_STAMPS")
ref = None
for name, env in variants:
    for k in keys:
        os.environ.pop(k, None)
    os.environ.update(env)
    plan = ops.execution_plan(mdp, "backward")
    pi = ops.backward_maxent(mdp, r, tm); torch.cuda.synchronize()   # warm
    t = time.perf_counter(); pi = ops.backward_maxent(mdp, r, tm); torch.cuda.synchronize()
    dt = time.perf_counter() - t
    same = ref is None or torch.equal(pi, ref)
    ref = pi if ref is None else ref
    print(f"{name}: {dt * 1e3:.1f} ms  plan R={plan['R']} G={plan['G']} C={plan['C']} spt={plan['spt']} "
          f"layout={plan['layout']} launches={plan['launches']}  bit-identical={same}", flush=True)
    os.environ["IRLMX_STAMPS"] = "1"
    ops.backward_maxent(mdp, r, tm); torch.cuda.synchronize()
