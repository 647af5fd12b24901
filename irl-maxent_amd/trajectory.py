"""Drop-in for the reference's ``trajectory.py`` (trajectories and expert demonstrations).

Same names, signatures and results as narendasan/irl-maxent ``src/trajectory.py``
(``Trajectory`` trajectory.py:10-49, ``generate_trajectory`` :52-85,
``generate_trajectories`` :88-128, ``policy_adapter`` :131-145,
``stochastic_policy_adapter`` :148-166), including the random draws: for the
same numpy global RNG state the generated trajectories are identical, draw for
draw, to the reference's (pinned by tests/golden/config1.npz, 200 trajectories
with ``np.random.seed(0)``).

The reference draws each successor with ``np.random.choice(range(S),
p=P[s, :, a])``, which builds the cumulative sum of all S probabilities per
step -- O(S) work and an O(S^2 A) dense table that cannot be built at 128x128.
Here the draw runs over the row's nonzeros only: the running sum over a row
with its zeros removed has the same values at the nonzero positions (adding
an exact zero changes nothing), the same total, and ``searchsorted(u,
'right')`` can only land on a nonzero position, so one ``random_sample()`` per
step selects the same successor.  Worlds may be the reference's (dense
``p_transition``) or an ``irlmx.DeviceMDP`` (stencil / ELL tables, copied to
the host once): O(1) per step at any grid size.
"""

from itertools import chain

import numpy as np


class Trajectory:
    """A trajectory of ``(state_from, action, state_to)`` transitions (trajectory.py:10-49)."""

    def __init__(self, transitions):
        self._t = transitions

    def transitions(self):
        return self._t

    def states(self):
        """Visited states in order, the final state included (trajectory.py:38-46)."""
        return map(lambda x: x[0], chain(self._t, [(self._t[-1][2], 0, 0)]))

    def __repr__(self):
        return "Trajectory({})".format(repr(self._t))

    def __str__(self):
        return "{}".format(self._t)


# -- successor rows --------------------------------------------------------------

class _Rows:
    """Per (state, action): successor states in ascending order and their
    probabilities, zeros removed."""

    def __init__(self, world):
        self.n_states = int(world.n_states)
        self._dense = None
        self._tgt = self._val = None
        p = getattr(world, "p_transition", None)
        if p is not None:
            self._dense = p
            return
        from irlmx import _lib  # an irlmx.DeviceMDP
        val = world.row_val.detach().cpu().numpy()[0]            # [A][K][S] (instance 0)
        S, W = self.n_states, int(world.width)
        s = np.arange(S)
        if world.layout == _lib.LAYOUT_STENCIL5:
            x, y = s % W, s // W
            H = S // W
            # stencil slots self, +x, -x, +y, -y (common.h stencil_nbr); off-grid slots
            # point at s itself and carry weight 0
            nbr = np.stack([s, np.where(x + 1 < W, s + 1, s), np.where(x > 0, s - 1, s),
                            np.where(y + 1 < H, s + W, s), np.where(y > 0, s - W, s)])
        else:
            nbr = world.row_idx.detach().cpu().numpy()[0].astype(np.int64)  # [K][S]
        self._tgt = nbr                                          # [K][S]
        self._val = val                                          # [A][K][S]

    def row(self, state, action):
        if self._dense is not None:
            r = self._dense[state, :, action]
            nz = np.flatnonzero(r)
            return nz, r[nz]
        t = self._tgt[:, state]
        v = self._val[action, :, state]
        keep = v != 0.0
        t, v = t[keep], v[keep]
        order = np.argsort(t, kind="stable")
        return t[order], v[order]


_cache = {}


def _rows(world):
    key = id(world)
    hit = _cache.get(key)
    if hit is None or hit[0] is not world:
        hit = (world, _Rows(world))
        _cache.clear()
        _cache[key] = hit
    return hit[1]


def _choice_sparse(idx, p):
    """``np.random.choice(range(S), p=dense_row)`` on the row's nonzeros: the same
    single ``random_sample()`` and the same selected index (see module docstring)."""
    if np.any(p < 0):
        raise ValueError("probabilities are not non-negative")
    if abs(float(np.sum(p)) - 1.0) > np.sqrt(np.finfo(np.float64).eps):
        raise ValueError("probabilities do not sum to 1")
    cdf = p.cumsum()
    cdf /= cdf[-1]
    u = np.random.random_sample()
    return idx[cdf.searchsorted(u, side="right")]


# -- generation --------------------------------------------------------------------

def generate_trajectory(world, policy, start, final):
    """One trajectory from ``start`` until a state in ``final`` (trajectory.py:52-85)."""
    rows = _rows(world)
    state = start
    trajectory = []
    while state not in final:
        action = policy(state)
        next_s, next_p = rows.row(state, action)
        next_state = _choice_sparse(next_s, next_p)
        trajectory += [(state, action, next_state)]
        state = next_state
    return Trajectory(trajectory)


def generate_trajectories(n, world, policy, start, final):
    """A generator of ``n`` trajectories (trajectory.py:88-128).  ``start``: a state,
    a list of states (chosen uniformly), or a distribution over all states."""
    start_states = np.atleast_1d(start)

    def _generate_one():
        if len(start_states) == world.n_states:
            s = np.random.choice(range(world.n_states), p=start_states)
        else:
            s = np.random.choice(start_states)
        return generate_trajectory(world, policy, s, final)

    return (_generate_one() for _ in range(n))


def policy_adapter(policy):
    """Deterministic policy array -> ``state -> action`` (trajectory.py:131-145)."""
    return lambda state: policy[state]


def stochastic_policy_adapter(policy):
    """Stochastic policy ``[state, action]`` -> sampled ``state -> action`` (trajectory.py:148-166)."""
    return lambda state: np.random.choice([*range(policy.shape[1])], p=policy[state, :])
