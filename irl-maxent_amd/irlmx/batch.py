"""Batched MaxEnt IRL: B independent gridworld instances per device call.

One ``step()`` is one gradient step of ``maxent.irl`` (maxent.py:240-252) for
every instance at once, entirely on the device:

    reward = theta                         (identity features, maxent.py:244)
    pi     = backward(reward)              (maxent.py:119-159, 2*S sweeps)
    svf    = forward(p0, pi)               (maxent.py:63-114, until max|dd| <= eps)
    grad   = e_features - svf              (maxent.py:248)
    theta *= exp(lr_k * grad)              (ExpSga + linear_decay, optimizer.py:154-167, 217-240)

No host round trip happens inside a step except the forward pass's own
convergence polling on the sweep shape.
"""

import torch

from . import ops
from .mdp import DeviceMDP


class BatchedMaxEnt:
    def __init__(self, mdp: DeviceMDP, e_features, p_initial, terminal, lr0=0.2, eps_esvf=1e-5,
                 theta0=1.0, rescale=True):
        self.mdp = mdp
        dev = mdp.device
        B, S = mdp.batch, mdp.n_states
        self.e_features = torch.as_tensor(e_features, dtype=torch.float64, device=dev).reshape(B, S)
        self.p_initial = torch.as_tensor(p_initial, dtype=torch.float64, device=dev).reshape(B, S)
        self.terminal = ops.terminal_mask(terminal, S, batch=B, device=dev)
        self.theta = torch.full((B, S), float(theta0), dtype=torch.float64, device=dev)
        self.lr0 = lr0
        self.eps_esvf = eps_esvf
        self.rescale = rescale
        self.k = 0
        self.last_forward_sweeps = None
        self.last_delta = None

    def lr(self, k):
        return self.lr0 / (1.0 + float(k))   # linear_decay(lr0, 1, 1)

    def backward(self):
        return ops.backward_maxent(self.mdp, self.theta, self.terminal, rescale=self.rescale)

    def forward(self, pi):
        return ops.forward_svf(self.mdp, self.p_initial, self.terminal, pi, self.eps_esvf)

    def update(self, svf):
        grad = self.e_features - svf
        old = self.theta.clone()
        self.theta.mul_(torch.exp(self.lr(self.k) * grad))
        self.k += 1
        self.last_delta = (self.theta - old).abs().amax(dim=1)   # maxent.py:252, per instance
        return grad

    def step(self):
        pi = self.backward()
        svf, iters, _ = self.forward(pi)
        self.last_forward_sweeps = iters
        self.update(svf)
        return svf
