"""Config 1 (src/main.py, 5x5): wall time of the drop-in maxent.irl / irl_causal
full runs (reference: 0.71-1.25 s and 7.2-12.8 s on the survey VM)
and of the batched device driver on the same problem."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import torch
import maxent as M
import maxent_oracle as O
from conftest import load_golden, unpack_trajectories
from irlmx import DeviceMDP
from irlmx.batch import BatchedMaxEnt

z = load_golden("config1")
P, tjs, feats = z["p_transition"], unpack_trajectories(z["traj_flat"], z["traj_lens"]), np.identity(25)
for name, fn in (("irl", lambda o: M.irl(P, feats, [24], tjs, o, O.Constant(1.0))),
                 ("irl_causal", lambda o: M.irl_causal(P, feats, [24], tjs, o, O.Constant(1.0), 0.7))):
    fn(O.ExpSga(lr=O.linear_decay(0.2)))
    t = time.perf_counter(); o = O.ExpSga(lr=O.linear_decay(0.2)); fn(o); dt = time.perf_counter() - t
    print(f"drop-in {name}: {o.k} steps in {dt:.3f} s ({o.k / dt:.0f} steps/s)", flush=True)
dev = torch.device("cuda", 0)
mdp = DeviceMDP.icy_gridworld(5, 0.2, device=dev)
for causal in (False, True):
    irl = BatchedMaxEnt(mdp, z["e_features"][None], z["p_initial"][None], [24], causal=causal,
                        discount=0.7 if causal else None)
    irl.run(eps=1e-4)
    irl = BatchedMaxEnt(mdp, z["e_features"][None], z["p_initial"][None], [24], causal=causal,
                        discount=0.7 if causal else None)
    torch.cuda.synchronize(); t = time.perf_counter(); r, k = irl.run(eps=1e-4); torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print(f"batched {'irl_causal' if causal else 'irl'}: {int(k[0])} steps in {dt:.3f} s ({int(k[0]) / dt:.0f} steps/s)")
