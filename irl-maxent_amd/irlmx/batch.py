"""Batched MaxEnt / MaxCausalEnt IRL: B independent gridworld instances per device call.

One ``step()`` is one gradient step of ``maxent.irl`` (maxent.py:240-252) or
``maxent.irl_causal`` (maxent.py:437-450) for every still-active instance at
once, entirely on the device:

    reward = F . theta                       (maxent.py:244 / 441)
    pi     = backward(reward)                (maxent.py:119-159, 2*S sweeps; causal:
                                              soft VI maxent.py:279-341)
    svf    = forward(p0, pi)                 (maxent.py:63-114, until max|dd| <= eps)
    grad   = e_features - F^T . svf          (maxent.py:248 / 445)
    theta  = optimizer(theta, grad, k)       (default ExpSga + linear_decay, optimizer.py:154-167,
                                              217-240; any of irlmx.optim's Sga, ExpSga,
                                              NormalizeGrad with the reference's schedules)

``F`` is the identity (``features=None``, the configs' case: reward = theta),
one ``[S, F]`` matrix shared by all instances, or ``[B, S, F]``.  ``run()``
repeats steps until every instance has met the reference's stopping rule
``max|theta_old - theta| <= eps`` (a NaN delta stops, as ``while NaN > eps``
does); a stopped instance's theta is frozen, so each instance ends exactly
where its own reference loop would.

Compaction (``run(compact=True)``, the default): once an instance has
stopped, the following steps run only the still-active instances -- their
tables, demonstration statistics and theta are gathered into a smaller batch
(``DeviceMDP.take``) and the kernels re-plan for it (fewer instances: more
CUs per instance) -- so a stopped instance no longer pays its 2*S backward
sweeps and its forward pass every step.  Per-instance results do not depend on
the batch they run in (every kernel shape and plan performs the same float64
operations in the same order per instance), so a compacted run equals an
uncompacted one bit for bit with identity features on the STENCIL5 and ELL
layouts (tests/test_gpu_full_run.py).  Two exceptions change rounding, not
results beyond it: with a feature matrix the F . theta / F^T . svf products are
torch GEMMs whose summation order may change with the batch size, and on the
DENSE layout the planner picks the GEMM or streaming kernel, the GEMM's
split-K waves and the dense-grid row blocking from the working batch, each with
its own per-row summation order (tested to 1e-9 against the uncompacted run).

No host round trip happens inside a step except the forward pass's own
convergence polling on the per-sweep shape.
"""

import numpy as np
import torch

from . import ops
from .mdp import DeviceMDP
from .optim import ExpSga, linear_decay


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
                 eps_esvf=1e-5, theta0=1.0, rescale=True, causal=False, discount=None, eps_lap=1e-5,
                 optimizer=None):
        """``theta0``: a float (the reference's Constant init, optimizer.py:369-398) or
        an array [F] or [B, F] (e.g. drawn with the reference's Uniform init,
        optimizer.py:334-366).  ``optimizer``: an irlmx.optim optimiser (default
        ExpSga(linear_decay(lr0)), the reference main.py's choice)."""
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
        self.phi = None
        if causal:
            if discount is None:
                raise ValueError("causal IRL needs a discount (maxent.py:383)")
            self.phi = terminal_reward(terminal, S, batch=B, device=dev)
        self.discount = discount
        self.eps_lap = eps_lap
        if np.ndim(theta0) == 0:
            self.theta = torch.full((B, n_f), float(theta0), dtype=torch.float64, device=dev)
        else:
            t0 = torch.as_tensor(np.asarray(theta0, dtype=np.float64), device=dev)
            self.theta = t0.expand(B, n_f).clone() if t0.dim() == 1 else t0.reshape(B, n_f).clone()
        self.lr0 = lr0
        self.optimizer = optimizer if optimizer is not None else ExpSga(linear_decay(lr0))
        self.eps_esvf = eps_esvf
        self.rescale = rescale
        self.k = 0
        self.active = torch.ones(B, dtype=torch.bool, device=dev)
        self.steps = torch.zeros(B, dtype=torch.int64, device=dev)
        self.last_forward_sweeps = None    # [B] int64, 0 for instances not computed in the last step
        self.last_backward_sweeps = None   # causal: soft VI sweeps of the last backward() [B]
        self.last_delta = None
        self._work = None                  # compacted working set (compact()), None = all instances

    @property
    def batch(self):
        return self.mdp.batch

    @property
    def working_batch(self):
        """Instances the next step computes (all, or the active ones after compact())."""
        return self.batch if self._work is None else int(self._work["idx"].numel())

    # -- working set ----------------------------------------------------------

    def compact(self):
        """Restrict the following steps to the instances that are still active.

        Gathers their tables, demonstration statistics, masks and features into a
        smaller batch; theta stays full size (the working rows are gathered and
        scattered per step).  Returns the working batch size."""
        idx = torch.nonzero(self.active).squeeze(1)
        n = int(idx.numel())
        if n == self.working_batch:
            return n
        sel = lambda t: t.index_select(0, idx).contiguous() if t is not None else None
        feats = self.features
        if feats is not None and feats.dim() == 3:
            feats = sel(feats)
        self._work = {"idx": idx, "mdp": self.mdp.take(idx), "e_features": sel(self.e_features),
                      "p_initial": sel(self.p_initial), "terminal": sel(self.terminal), "phi": sel(self.phi),
                      "features": feats, "active": torch.ones(n, dtype=torch.bool, device=idx.device)}
        return n

    def _w(self, name):
        if self._work is None:
            return getattr(self, name)
        return self._work[name]

    def _theta_w(self):
        return self.theta if self._work is None else self.theta.index_select(0, self._work["idx"])

    def _active_w(self):
        return self.active if self._work is None else self.active.index_select(0, self._work["idx"])

    def _scatter(self, vec_w, fill=0):
        """A per-instance vector of the working set, expanded to all B instances."""
        if self._work is None:
            return vec_w
        out = torch.full((self.batch,) + tuple(vec_w.shape[1:]), fill, dtype=vec_w.dtype, device=vec_w.device)
        out[self._work["idx"]] = vec_w
        return out

    # -- one gradient step --------------------------------------------------

    def reward(self, theta=None, features=None):
        """F . theta (maxent.py:244): [B, S] for all instances by default."""
        if theta is None:
            theta, features = self.theta, self.features
        if features is None:
            return theta
        if features.dim() == 2:
            return theta @ features.T
        return torch.bmm(features, theta.unsqueeze(2)).squeeze(2)

    def features_t(self, svf, features=None):
        """F^T . svf, [n, F] (maxent.py:248)."""
        if features is None:
            features = self._w("features")
        if features is None:
            return svf
        if features.dim() == 2:
            return svf @ features
        return torch.bmm(svf.unsqueeze(1), features).squeeze(1)

    def backward(self):
        """Policy [n, S, A] of the working set (maxent.py:119-159 / 279-341)."""
        r = self.reward(self._theta_w(), self._w("features"))
        mdp = self._w("mdp")
        if self.causal:
            pi, _, k, _ = ops.soft_backward(mdp, r, self._w("phi"), self.discount, self.eps_lap)
            self.last_backward_sweeps = self._scatter(k)
            return pi
        return ops.backward_maxent(mdp, r, self._w("terminal"), rescale=self.rescale)

    def forward(self, pi):
        """``(svf [n, S], sweeps [n], status [n])`` of the working set (maxent.py:63-114)."""
        return ops.forward_svf(self._w("mdp"), self._w("p_initial"), self._w("terminal"), pi, self.eps_esvf)

    def update(self, svf):
        """Optimiser step on the working set's theta (default ExpSga,
        optimizer.py:154-167); stopped instances stay frozen.  Returns the gradient [n, F]."""
        theta = self._theta_w()
        act = self._active_w()
        grad = self._w("e_features") - self.features_t(svf)
        new = self.optimizer.apply(theta, grad, self.k)
        delta = torch.where(act, (new - theta).abs().amax(dim=1),
                            torch.zeros((), dtype=torch.float64, device=theta.device))
        new = torch.where(act.unsqueeze(1), new, theta)
        if self._work is None:
            self.theta = new
        else:
            self.theta[self._work["idx"]] = new
        self.last_delta = self._scatter(delta)
        self.steps += self.active.to(torch.int64)
        self.k += 1
        return grad

    def step(self):
        pi = self.backward()
        svf, iters, _ = self.forward(pi)
        self.last_forward_sweeps = self._scatter(iters)
        self.update(svf)
        return svf

    def prime_compaction(self, eps=1e-4):
        """Run, once, every device operation of ``run()`` outside the passes --
        the stop test, ``compact()`` and ``update()`` on a working set, the
        scatter of its results -- on a scratch copy of this object (its state is
        left unchanged), for working sets of more and of at most 16 instances
        (torch's index_select switches kernels at 16 indices).  The first use of
        a device kernel in a process pays its code-object load: without this,
        bench.py's full run paid ~0.13 s at its first step and ~0.13 s at the
        first compaction to 15 instances (tools/diag/full_run_steps.py)."""
        import copy
        B = self.batch
        dev = self.theta.device
        for n in sorted({n for n in (B - 1, min(B - 1, 16), 1) if n >= 1}, reverse=True):
            sc = copy.copy(self)
            sc.theta, sc.steps, sc._work = self.theta.clone(), self.steps.clone(), None
            sc.active = torch.zeros(B, dtype=torch.bool, device=dev)
            sc.active[:n] = True
            sc.compact()
            svf = torch.zeros((n, self.mdp.n_states), dtype=torch.float64, device=dev)
            sc.last_forward_sweeps = sc._scatter(torch.zeros(n, dtype=torch.int64, device=dev))
            sc.update(svf)
            sc.active &= sc.last_delta > eps
            bool(sc.active.any())
            sc.reward()
        torch.cuda.synchronize(dev)

    def run(self, eps=1e-4, max_steps=None, compact=True, on_step=None):
        """Step until every instance meets ``max|dtheta| <= eps`` (maxent.py:240, 252).

        ``compact``: drop stopped instances from the working set before each
        step (module docstring).  ``on_step(self)`` is called after every step.
        Returns ``(reward [B, S], steps [B])`` -- ``features . theta`` and the
        number of gradient steps each instance took.
        """
        while bool(self.active.any()):
            if max_steps is not None and self.k >= max_steps:
                break
            if compact:
                self.compact()
            self.step()
            self.active &= self.last_delta > eps   # NaN > eps is False: a NaN step stops
            if on_step is not None:
                on_step(self)
        return self.reward(), self.steps
