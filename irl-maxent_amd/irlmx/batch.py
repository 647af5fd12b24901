"""Batched MaxEnt / MaxCausalEnt IRL: B independent gridworld instances per device call.

One ``step()`` is one gradient step of ``maxent.irl`` (maxent.py:240-252) or
``maxent.irl_causal`` (maxent.py:437-450) for every still-active instance at
once, entirely on the device:

    reward = F . theta                       (maxent.py:244 / 441)
    pi     = backward(reward)                (maxent.py:119-159, 2*S sweeps; causal:
                                              soft VI maxent.py:279-341)
    svf    = forward(p0, pi)                 (maxent.py:63-114, until max|dd| <= eps)
    grad   = e_features - F^T . svf          (maxent.py:248 / 445)
    theta *= exp(lr_k * grad)                (ExpSga + linear_decay, optimizer.py:154-167, 217-240)

``F`` is the identity (``features=None``, the configs' case: reward = theta),
one ``[S, F]`` matrix shared by all instances, or ``[B, S, F]``.  ``run()``
repeats steps until every instance has met the reference's stopping rule
``max|theta_old - theta| <= eps`` (a NaN delta stops, as ``while NaN > eps``
does); a stopped instance's theta is frozen, so each instance ends exactly
where its own reference loop would.

No host round trip happens inside a step except the forward pass's own
convergence polling on the per-sweep shape.
"""

import numpy as np
import torch

from . import ops
from .mdp import DeviceMDP


def terminal_reward(terminal, n_states, batch=1, device=None):
    """phi of the causal backward pass (maxent.py:313-317), as float64 [B, S]:
    0 at the terminal states and -inf elsewhere, or ``terminal`` itself when it
    has one entry per state."""
    if len(terminal) == n_states:
        phi = np.array(terminal, dtype=float)
    else:
        phi = -np.inf * np.ones(n_states)
        phi[terminal] = 0.0
    return torch.as_tensor(np.tile(phi, (batch, 1)), dtype=torch.float64, device=device)


class BatchedMaxEnt:
    def __init__(self, mdp: DeviceMDP, e_features, p_initial, terminal, features=None, lr0=0.2,
                 eps_esvf=1e-5, theta0=1.0, rescale=True, causal=False, discount=None, eps_lap=1e-5):
        self.mdp = mdp
        dev = mdp.device
        B, S = mdp.batch, mdp.n_states
        if features is None:
            self.features = None
            n_f = S
        else:
            f = torch.as_tensor(features, dtype=torch.float64, device=dev)
            if f.dim() == 2:
                assert f.shape[0] == S, f.shape
            else:
                assert f.dim() == 3 and f.shape[:2] == (B, S), f.shape
            self.features = f
            n_f = f.shape[-1]
        self.e_features = torch.as_tensor(e_features, dtype=torch.float64, device=dev).reshape(B, n_f)
        self.p_initial = torch.as_tensor(p_initial, dtype=torch.float64, device=dev).reshape(B, S)
        self.terminal = ops.terminal_mask(terminal, S, batch=B, device=dev)
        self.causal = causal
        if causal:
            if discount is None:
                raise ValueError("causal IRL needs a discount (maxent.py:383)")
            self.phi = terminal_reward(terminal, S, batch=B, device=dev)
        self.discount = discount
        self.eps_lap = eps_lap
        self.theta = torch.full((B, n_f), float(theta0), dtype=torch.float64, device=dev)
        self.lr0 = lr0
        self.eps_esvf = eps_esvf
        self.rescale = rescale
        self.k = 0
        self.active = torch.ones(B, dtype=torch.bool, device=dev)
        self.steps = torch.zeros(B, dtype=torch.int64, device=dev)
        self.last_forward_sweeps = None
        self.last_backward_sweeps = None   # causal: soft VI sweeps of the last backward() [B]
        self.last_delta = None

    def lr(self, k):
        return self.lr0 / (1.0 + float(k))   # linear_decay(lr0, 1, 1)

    def reward(self):
        """F . theta, [B, S] (maxent.py:244)."""
        if self.features is None:
            return self.theta
        if self.features.dim() == 2:
            return self.theta @ self.features.T
        return torch.bmm(self.features, self.theta.unsqueeze(2)).squeeze(2)

    def features_t(self, svf):
        """F^T . svf, [B, F] (maxent.py:248)."""
        if self.features is None:
            return svf
        if self.features.dim() == 2:
            return svf @ self.features
        return torch.bmm(svf.unsqueeze(1), self.features).squeeze(1)

    def backward(self):
        r = self.reward()
        if self.causal:
            pi, _, k, _ = ops.soft_backward(self.mdp, r, self.phi, self.discount, self.eps_lap)
            self.last_backward_sweeps = k
            return pi
        return ops.backward_maxent(self.mdp, r, self.terminal, rescale=self.rescale)

    def forward(self, pi):
        return ops.forward_svf(self.mdp, self.p_initial, self.terminal, pi, self.eps_esvf)

    def update(self, svf):
        grad = self.e_features - self.features_t(svf)
        new = self.theta * torch.exp(self.lr(self.k) * grad)
        act = self.active.unsqueeze(1)
        self.last_delta = torch.where(self.active, (new - self.theta).abs().amax(dim=1),
                                      torch.zeros((), dtype=torch.float64, device=self.theta.device))
        self.theta = torch.where(act, new, self.theta)   # stopped instances stay frozen
        self.steps += self.active.to(torch.int64)
        self.k += 1
        return grad

    def step(self):
        pi = self.backward()
        svf, iters, _ = self.forward(pi)
        self.last_forward_sweeps = iters
        self.update(svf)
        return svf

    def run(self, eps=1e-4, max_steps=None):
        """Step until every instance meets ``max|dtheta| <= eps`` (maxent.py:240, 252).

        Returns ``(reward [B, S], steps [B])`` -- ``features . theta`` and the
        number of gradient steps each instance took.
        """
        while bool(self.active.any()):
            if max_steps is not None and self.k >= max_steps:
                break
            self.step()
            self.active &= self.last_delta > eps   # NaN > eps is False: a NaN step stops
        return self.reward(), self.steps
