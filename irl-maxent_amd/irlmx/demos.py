"""Synthetic expert demonstrations for gridworld instances (bench / test inputs).

The reference samples demonstrations one step at a time with
``np.random.choice`` over all S states (trajectory.py:52-128), which is O(S)
per step.  This generator samples ``n`` trajectories in lock-step with numpy,
drawing each successor from the <= 5 stencil targets of the STENCIL5 table,
and returns the two statistics the IRL loop consumes (maxent.py:15-60):
the visit-count feature expectation (final states included) and the
start-state distribution.  It is input generation, outside any timed region.

Expert: a stochastic policy that prefers actions whose intended successor is
closer (Manhattan distance) to the goal, p(a|s) ~ exp(-beta * dist).
"""

import numpy as np

_DX = np.array([1, -1, 0, 0])
_DY = np.array([0, 0, 1, -1])


def expert_policy(size, goal, beta=2.0):
    s = np.arange(size * size)
    x, y = s % size, s // size
    gx, gy = goal % size, goal // size
    logits = np.empty((size * size, 4))
    for a in range(4):
        nx = np.clip(x + _DX[a], 0, size - 1)
        ny = np.clip(y + _DY[a], 0, size - 1)
        logits[:, a] = -beta * (np.abs(nx - gx) + np.abs(ny - gy))
    logits -= logits.max(axis=1, keepdims=True)
    p = np.exp(logits)
    return p / p.sum(axis=1, keepdims=True)


def stencil_targets(size):
    """[S, 5] target state of each stencil slot (self, +x, -x, +y, -y); -1 off-grid."""
    s = np.arange(size * size)
    x, y = s % size, s // size
    return np.stack([s, np.where(x + 1 < size, s + 1, -1), np.where(x > 0, s - 1, -1),
                     np.where(y + 1 < size, s + size, -1), np.where(y > 0, s - size, -1)], axis=1)


def safety_cap(size):
    """A step cap for callers that must not hang on a trajectory that can never
    reach a terminal state (bench.py, the tests): 64 x the grid side, far above
    any expert trajectory of these worlds (a cut raises by default)."""
    return 64 * size


class TruncatedDemonstrations(ValueError):
    """Some trajectories were cut at ``max_len`` before reaching a terminal state."""


def sample(row_val, size, terminal, start, n=200, seed=0, beta=2.0, max_len=None, on_truncate="raise",
           with_truncated=False):
    """Sample ``n`` demonstrations on one STENCIL5 table ``row_val`` [4, 5, S].

    Like the reference (trajectory.py:76, ``while not terminal``) a trajectory
    runs until it reaches a terminal state: with ``max_len=None`` there is no
    cap, so the caller must guarantee that terminals are reachable (bench.py
    and the tests pass ``max_len=safety_cap(size)``).  With a cap, trajectories still alive after ``max_len`` steps are cut
    (their last state then counts as a final state, which skews the feature
    expectation): ``on_truncate="raise"`` raises TruncatedDemonstrations,
    ``"allow"`` keeps them.  Returns ``(e_features, p_initial, lengths)`` for
    identity state features, plus the number of cut trajectories when
    ``with_truncated``.
    """
    if on_truncate not in ("raise", "allow"):
        raise ValueError(f"on_truncate must be 'raise' or 'allow', got {on_truncate!r}")
    rng = np.random.default_rng(seed)
    S = size * size
    goal = terminal[0]
    pol = np.cumsum(expert_policy(size, goal, beta), axis=1)
    tgt = stencil_targets(size)
    trans = np.cumsum(np.transpose(row_val, (2, 0, 1)), axis=2)   # [S, A, 5]
    is_term = np.zeros(S, dtype=bool)
    is_term[terminal] = True
    state = np.full(n, start, dtype=np.int64)
    counts = np.zeros(S)
    p_init = np.bincount(state, minlength=S) / n
    alive = ~is_term[state]
    lengths = np.zeros(n, dtype=np.int64)
    steps = 0
    while alive.any():
        if max_len is not None and steps >= max_len:
            break
        idx = np.nonzero(alive)[0]
        s = state[idx]
        np.add.at(counts, s, 1.0)
        a = (rng.random(len(idx))[:, None] > pol[s]).sum(axis=1).clip(0, 3)
        cdf = trans[s, a]                                          # [m, 5]
        k = (rng.random(len(idx))[:, None] * cdf[:, -1:] > cdf).sum(axis=1).clip(0, 4)
        nxt = tgt[s, k]
        nxt = np.where(nxt < 0, s, nxt)
        state[idx] = nxt
        lengths[idx] += 1
        alive[idx] = ~is_term[nxt]
        steps += 1
    truncated = int(np.count_nonzero(alive))
    if truncated and on_truncate == "raise":
        raise TruncatedDemonstrations(f"{truncated} of {n} demonstrations did not reach a terminal state within "
                                      f"max_len={max_len} steps (the reference samples until terminal)")
    np.add.at(counts, state, 1.0)                                  # final states (trajectory.py:43)
    out = (counts / n, p_init, lengths)
    return out + (truncated,) if with_truncated else out
