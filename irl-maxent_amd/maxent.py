"""MI355X drop-in for the reference module ``maxent`` (narendasan/irl-maxent, src/maxent.py).

Same public names, signatures, defaults and return types (float64 numpy
arrays) as the reference, so ``src/main.py`` runs unchanged with this
directory ahead of ``src/`` on ``sys.path``.  The fixed-point loops run on the
GPU through libirlmx.so (``irlmx.ops``); only the demonstration statistics,
the feature products and the user's optimizer stay on the host, as in the
reference's outer loop.

The backward passes run in numpy's own floating-point order when the model
allows it (S % 4 in {0, 1}: every square grid; by default up to 1024 states for
the backward and forward, 4096 for soft VI, 64 on a DENSE table --
ops.numpy_order_default): the non-causal
policy (local_action_probabilities, and the backward half of
compute_expected_svf / irl) is then bit-identical to the reference's on a
Haswell-family OpenBLAS host, and the soft VI's dot products follow numpy's
order (ops.*_numpy_order; IRLMX_NUMPY_ORDER=0 turns it off).
Above 625 states that is the reference run with one BLAS thread
(OPENBLAS_NUM_THREADS=1): numpy's multi-threaded OpenBLAS partitions the rows
differently there and its own last bits move with the thread count.

Deliberate differences (documented in DESIGN.md):
* Where the reference's backward pass overflows to NaN (about 13x13 at unit
  reward) the drop-in reruns it with its partition vector rescaled by powers
  of two (ratio-exact), so the policy stays finite.
  ``IRLMX_REFERENCE_OVERFLOW=1`` keeps the reference's NaN instead.
* ``p_transition`` may also be an ``irlmx.DeviceMDP`` already resident in HBM.
"""

import os
from itertools import chain

import numpy as np
import torch

from irlmx import DeviceMDP, ops

__all__ = ["feature_expectation_from_trajectories", "initial_probabilities_from_trajectories",
           "expected_svf_from_policy", "local_action_probabilities", "compute_expected_svf",
           "expected_svf", "irl", "softmax", "local_causal_action_probabilities",
           "compute_expected_causal_svf", "irl_causal"]


def _rescale():
    return os.environ.get("IRLMX_REFERENCE_OVERFLOW", "0") != "1"


def _model(p_transition):
    """The device model of ``p_transition`` (uploaded once per array, see
    DeviceMDP.resident; the reference re-copies it per call, maxent.py:98-102, 143, 320)."""
    if isinstance(p_transition, DeviceMDP):
        return p_transition
    return DeviceMDP.resident(p_transition)


def _host(t):
    return t[0].detach().cpu().numpy()


def _fdot(features, x, ident, transpose=False):
    # identity features: F.x == x bit for bit while x is finite (0 * finite adds
    # exact zeros); a non-finite x takes the real product so NaN spreads as in numpy
    if ident and np.isfinite(x).all():
        return x.copy()
    return features.T.dot(x) if transpose else features.dot(x)


def _is_identity(features):
    n, f = features.shape
    if n != f:
        return False
    return bool(np.all(np.diagonal(features) == 1.0)) and int(np.count_nonzero(features)) == n


# -- demonstration statistics (host, once per IRL run) -------------------------

def feature_expectation_from_trajectories(features, trajectories):
    """Average feature vector over all visited states, final states included (maxent.py:15-39)."""
    n_states, n_features = features.shape
    visited = np.fromiter(chain.from_iterable(t.states() for t in trajectories), dtype=np.int64)
    if np.array_equal(features, np.round(features)):
        # integer-valued features: visit counts times features is exact, so the
        # result equals the reference's sequential sum bit for bit
        counts = np.bincount(visited, minlength=n_states).astype(np.float64)
        fe = counts.dot(features)
    else:
        fe = np.zeros(n_features)
        for s in visited:
            fe += features[s, :]
    return fe / len(trajectories)


def initial_probabilities_from_trajectories(n_states, trajectories):
    """Fraction of trajectories starting in each state (maxent.py:42-60)."""
    p = np.zeros(n_states)
    for t in trajectories:
        p[t.transitions()[0][0]] += 1.0
    return p / len(trajectories)


# -- plain MaxEnt (Ziebart et al. 2008) -----------------------------------------

def expected_svf_from_policy(p_transition, p_initial, terminal, p_action, eps=1e-5):
    """Expected state visitation frequencies under ``p_action`` (maxent.py:63-114)."""
    mdp = _model(p_transition)
    term = ops.terminal_mask(terminal, mdp.n_states, device=mdp.device)
    svf, _, _ = _forward(mdp, p_initial, term, p_action, eps)
    return _host(svf)


def _np_order(mdp, op="backward"):
    """numpy's own summation order for this call: one instance of a model the
    numpy-order kernels cover, up to a per-op state count (backward / forward
    1024, soft VI 4096; 64 on a DENSE table) -- ops.numpy_order_default states
    the caps, their measured cost and the environment overrides
    (IRLMX_NUMPY_ORDER=0 turns it off)."""
    return ops.numpy_order_default(mdp, op)


def _forward(mdp, p_initial, term, pi, eps):
    return ops.forward_svf(mdp, p_initial, term, pi, eps, numpy_order=_np_order(mdp, "forward"))


def _backward(mdp, reward, term):
    """The backward policy on the device: numpy's order where the model allows it
    (bit-identical to the reference), the rescaled pass where that overflows
    (the numpy-order kernel stops at the overflow, so the detour costs the sweeps
    up to it: a few hundred at unit reward)."""
    reward = np.asarray(reward.cpu().numpy() if torch.is_tensor(reward) else reward, dtype=np.float64)
    if _np_order(mdp):
        pi = ops.backward_maxent_numpy_order(mdp, np.exp(reward), term)   # er = np.exp(reward), maxent.py:142
        if not _rescale() or bool(torch.isfinite(pi).all()):
            return pi
    return ops.backward_maxent(mdp, reward, term, rescale=_rescale())


def local_action_probabilities(p_transition, terminal, reward):
    """Backward pass of MaxEnt IRL, 2*S sweeps (maxent.py:119-159)."""
    mdp = _model(p_transition)
    term = ops.terminal_mask(terminal, mdp.n_states, device=mdp.device)
    return _host(_backward(mdp, reward, term))


def compute_expected_svf(p_transition, p_initial, terminal, reward, eps=1e-5):
    """Backward pass then forward pass (maxent.py:162-193)."""
    mdp = _model(p_transition)
    term = ops.terminal_mask(terminal, mdp.n_states, device=mdp.device)
    pi = _backward(mdp, reward, term)
    svf, _, _ = _forward(mdp, p_initial, term, pi, eps)
    return _host(svf)


expected_svf = compute_expected_svf


def _irl_loop(mdp, features, terminal, trajectories, optim, init, eps, svf_fn):
    n_states = mdp.n_states
    _, n_features = features.shape
    e_features = feature_expectation_from_trajectories(features, trajectories)
    p_initial = initial_probabilities_from_trajectories(n_states, trajectories)
    ident = _is_identity(features)
    term = ops.terminal_mask(terminal, n_states, device=mdp.device)
    p0 = torch.as_tensor(p_initial, device=mdp.device)

    theta = init(n_features)
    delta = np.inf
    optim.reset(theta)                       # theta is aliased and mutated by optim.step
    while delta > eps:
        theta_old = theta.copy()
        reward = _fdot(features, theta, ident)
        e_svf = svf_fn(mdp, reward, term, p0)
        grad = e_features - _fdot(features, e_svf, ident, transpose=True)
        optim.step(grad)
        delta = np.max(np.abs(theta_old - theta))
    return _fdot(features, theta, ident)


def irl(p_transition, features, terminal, trajectories, optim, init, eps=1e-4, eps_esvf=1e-5):
    """MaxEnt IRL by gradient ascent on the demonstration likelihood (maxent.py:196-255).

    The transition model is uploaded once; every gradient step runs the
    backward and forward passes on the device and moves only the reward (H2D)
    and the visitation frequencies (D2H) across PCIe.
    """
    mdp = _model(p_transition)

    def svf_fn(m, reward, term, p0):
        pi = _backward(m, reward, term)
        svf, _, _ = _forward(m, p0, term, pi, eps_esvf)
        return _host(svf)

    return _irl_loop(mdp, features, terminal, trajectories, optim, init, eps, svf_fn)


# -- maximum causal entropy (Ziebart 2010) -------------------------------------

def softmax(x1, x2):
    """Elementwise soft maximum max + log(1 + exp(min - max)) (maxent.py:260-276)."""
    x_max = np.maximum(x1, x2)
    x_min = np.minimum(x1, x2)
    return x_max + np.log(1.0 + np.exp(x_min - x_max))


def _terminal_reward(terminal, n_states):
    # maxent.py:313-317: a full-length `terminal` is the terminal reward itself
    if len(terminal) == n_states:
        return np.array(terminal, dtype=float)
    phi = -np.inf * np.ones(n_states)
    phi[terminal] = 0.0
    return phi


def local_causal_action_probabilities(p_transition, terminal, reward, discount, eps=1e-5):
    """Soft value iteration of MaxCausalEnt IRL; returns exp(Q - V) (maxent.py:279-341)."""
    mdp = _model(p_transition)
    phi = _terminal_reward(terminal, mdp.n_states)
    pi, _, _, _ = ops.soft_backward(mdp, reward, phi, discount, eps, numpy_order=_np_order(mdp, "soft_backward"))
    return _host(pi)


def compute_expected_causal_svf(p_transition, p_initial, terminal, reward, discount,
                                eps_lap=1e-5, eps_svf=1e-5):
    """Soft value iteration then forward pass (maxent.py:344-380)."""
    mdp = _model(p_transition)
    phi = _terminal_reward(terminal, mdp.n_states)
    pi, _, _, _ = ops.soft_backward(mdp, reward, phi, discount, eps_lap, numpy_order=_np_order(mdp, "soft_backward"))
    term = ops.terminal_mask(terminal, mdp.n_states, device=mdp.device)
    svf, _, _ = _forward(mdp, p_initial, term, pi, eps_svf)
    return _host(svf)


def irl_causal(p_transition, features, terminal, trajectories, optim, init, discount,
               eps=1e-4, eps_svf=1e-5, eps_lap=1e-5):
    """MaxCausalEnt IRL by gradient ascent (maxent.py:383-453)."""
    mdp = _model(p_transition)
    phi = torch.as_tensor(_terminal_reward(terminal, mdp.n_states), device=mdp.device)

    def svf_fn(m, reward, term, p0):
        pi, _, _, _ = ops.soft_backward(m, reward, phi, discount, eps_lap, numpy_order=_np_order(m, "soft_backward"))
        svf, _, _ = _forward(m, p0, term, pi, eps_svf)
        return _host(svf)

    return _irl_loop(mdp, features, terminal, trajectories, optim, init, eps, svf_fn)
