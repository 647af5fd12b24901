"""Per-step breakdown of config 3's whole irl run (bench.py full_run): for every
gradient step the compaction (host + device), backward, forward and update
times (each phase synchronised, wall clock) and the library's event counters;
prints the steps that take more than 1.3x the median of their neighbours.
usage: python tools/diag/full_run_steps.py [size B]"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import torch
from irlmx import DeviceMDP, demos, ops
from irlmx.batch import BatchedMaxEnt
from irlmx.shard import instance_slips

dev = torch.device("cuda", 0)
size = int(sys.argv[1]) if len(sys.argv) > 1 else 128
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
S = size * size
mdp = DeviceMDP.icy_gridworld(size, instance_slips(np.arange(B), B), device=dev)
rv = mdp.row_val.cpu().numpy()
e_f = np.empty((B, S))
p0 = np.empty((B, S))
for b in range(B):
    e_f[b], p0[b], _ = demos.sample(rv[b], size, [S - 1], 0, n=200, seed=1234 + b, max_len=demos.safety_cap(size))
prime = BatchedMaxEnt(mdp, e_f, p0, [S - 1])
svf_p, _, _ = ops.forward_svf(mdp, prime.p_initial, prime.terminal, prime.backward(), max_iter=16)
prime.update(svf_p)
prime.last_delta.cpu()
if os.environ.get("NO_PRIME_COMPACTION") != "1":
    prime.prime_compaction()
del prime, svf_p
torch.cuda.synchronize()

irl = BatchedMaxEnt(mdp, e_f, p0, [S - 1])
rec = []
t_start = time.perf_counter()
while bool(irl.active.any()):
    c0 = ops.counters()
    t0 = time.perf_counter()
    n = irl.compact()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    pi = irl.backward()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    svf, iters, _ = irl.forward(pi)
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    irl.last_forward_sweeps = irl._scatter(iters)
    irl.update(svf)
    irl.active &= irl.last_delta > 1e-4
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    c1 = ops.counters()
    rec.append((irl.k, n, (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, (t4 - t3) * 1e3, int(iters.max()),
                {k: c1[k] - c0[k] for k in c0 if c1[k] != c0[k]}))
wall = time.perf_counter() - t_start
tot = np.array([r[2] + r[3] + r[4] + r[5] for r in rec])
print(f"whole run {wall:.3f} s, {len(rec)} steps, {int(irl.steps.sum())} instance-steps", flush=True)
print("step batch compact_ms backward_ms forward_ms update_ms fwd_sweeps counters", flush=True)
for i, r in enumerate(rec):
    lo, hi = max(0, i - 3), min(len(rec), i + 4)
    nb = np.median(np.delete(tot[lo:hi], i - lo)) if hi - lo > 1 else tot[i]
    flag = " <-- outlier" if tot[i] > 1.3 * nb and i > 0 else ""
    if flag or i < 2 or (i > 0 and rec[i][1] != rec[i - 1][1]):
        print(f"{r[0]:4d} {r[1]:3d} {r[2]:8.2f} {r[3]:8.2f} {r[4]:8.2f} {r[5]:8.2f} {r[6]:7d} {r[7]}{flag}", flush=True)
