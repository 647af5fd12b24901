"""One warm-up and one measured backward pass for rocprofv3 counter passes on
the cluster kernel: config 3 (128x128, B = 64) by default, or
`python tools/diag/bwd_once.py SIZE B` (config 4: 256 32), the bench's slips."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "irl-maxent_amd")]
import torch
from irlmx import DeviceMDP, ops
from irlmx.shard import instance_slips
dev = torch.device("cuda", 0)
size = int(sys.argv[1]) if len(sys.argv) > 1 else 128
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
n = size * size
mdp = DeviceMDP.icy_gridworld(size, instance_slips(np.arange(B), B), device=dev)
tm = ops.terminal_mask([n - 1], n, batch=B, device=dev)
r = torch.ones((B, n), dtype=torch.float64, device=dev)
for _ in range(2):
    ops.backward_maxent(mdp, r, tm)
torch.cuda.synchronize()
print("done", ops.execution_plan(mdp, "backward"))
