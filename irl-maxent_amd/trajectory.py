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

import operator
from functools import partial

import numpy as np


class Trajectory:
    """A demonstration: a list of ``(state_from, action, state_to)`` transitions
    (the container of trajectory.py:10-49; the same accessors and string forms)."""

    __slots__ = ("_steps",)

    def __init__(self, transitions):
        self._steps = transitions

    def transitions(self):
        return self._steps

    def states(self):
        """Iterator over the visited states in order, the final state included
        (trajectory.py:33-43).  The final state is read at call time, so an empty
        trajectory raises IndexError here, as the reference's does."""
        final = self._steps[-1][2]

        def visits():
            for step in self._steps:
                yield step[0]
            yield final
        return visits()

    def __repr__(self):
        return f"Trajectory({self._steps!r})"

    def __str__(self):
        return str(self._steps)


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
    """One trajectory from ``start`` until a state in ``final`` (trajectory.py:52-87):
    per step one policy call, then one successor draw."""
    rows = _rows(world)
    steps = []
    state = start
    while state not in final:
        action = policy(state)
        succ = _choice_sparse(*rows.row(state, action))
        steps.append((state, action, succ))
        state = succ
    return Trajectory(steps)


def generate_trajectories(n, world, policy, start, final):
    """Lazily generate ``n`` trajectories (trajectory.py:90-128).  ``start``: one
    state, a list of states (one drawn uniformly per trajectory), or a
    distribution over all states (when it has one entry per state)."""
    starts = np.atleast_1d(start)

    def draw_start():
        if len(starts) == world.n_states:
            return np.random.choice(world.n_states, p=starts)   # same single draw as choice(range(S), p)
        return np.random.choice(starts)

    def trajectories():
        for _ in range(n):
            yield generate_trajectory(world, policy, draw_start(), final)
    return trajectories()


def policy_adapter(policy):
    """Deterministic policy (array or map ``state -> action``) as a callable
    (trajectory.py:131-147)."""
    return partial(operator.getitem, policy)


def stochastic_policy_adapter(policy):
    """Stochastic policy ``[state, action]`` as a callable that samples an action
    per call (trajectory.py:150-169)."""
    n_actions = policy.shape[1]
    return lambda state: np.random.choice(n_actions, p=policy[state, :])
