"""Time the bench's config-3 workload step by step (B = 64, 128x128), printing as it goes."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import numpy as np, torch
import irlmx
from irlmx import DeviceMDP, demos, ops
from irlmx.batch import BatchedMaxEnt
from irlmx.shard import instance_slips
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
size = 128; S = size * size
dev = torch.device("cuda", 0)
t = time.time()
mdp = DeviceMDP.icy_gridworld(size, instance_slips(np.arange(B), B), device=dev)
rv = mdp.row_val.cpu().numpy()
e_f = np.empty((B, S)); p0 = np.empty((B, S))
for b in range(B):
    e_f[b], p0[b], _ = demos.sample(rv[b], size, [S - 1], 0, n=200, seed=1234 + b, max_len=demos.safety_cap(size))
print("setup", time.time() - t, flush=True)
if hasattr(irlmx._lib.load(), "irlmx_execution_plan"):
    print("plans", ops.execution_plan(mdp, "backward"), ops.execution_plan(mdp, "forward"), flush=True)
irl = BatchedMaxEnt(mdp, e_f, p0, [S - 1])
for i in range(int(os.environ.get("STEPS", "3"))):
    t = time.time(); pi = irl.backward(); torch.cuda.synchronize(); tb = time.time() - t
    t = time.time(); svf, k, st = irl.forward(pi); torch.cuda.synchronize(); tf = time.time() - t
    irl.update(svf)
    print(f"step {i}: backward {tb*1e3:.1f} ms forward {tf*1e3:.1f} ms k_f[0]={int(k[0])} k_f[-1]={int(k[-1])} "
          f"st={st.max().item()} pi finite={bool(torch.isfinite(pi).all())}", flush=True)
