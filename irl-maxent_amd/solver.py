"""MI355X drop-in for the reference module ``solver`` (narendasan/irl-maxent, src/solver.py).

Value iteration runs as a device fixed-point loop (irlmx.ops.value_iteration),
in numpy's summation order where the model allows it (bit-identical values;
above 625 states to the reference run with OPENBLAS_NUM_THREADS=1, whose
multi-threaded row partition moves its own last bits);
policy extraction gathers the intended successors' values on the device.
Names, signatures, defaults and float64 numpy results follow the reference.
"""


import numpy as np
import torch

from irlmx import DeviceMDP, ops

__all__ = ["value_iteration", "stochastic_value_iteration", "optimal_policy_from_value",
           "optimal_policy", "stochastic_policy_from_value"]


def _model(p):
    return p if isinstance(p, DeviceMDP) else DeviceMDP.resident(p)


def _np_order(mdp):
    # numpy's summation order where the kernels cover the model: values bit-identical
    # to the reference's (ops.value_iteration numpy_order; caps and IRLMX_NUMPY_ORDER:
    # ops.numpy_order_default)
    return ops.numpy_order_default(mdp, "value_iteration")


def value_iteration(p, reward, discount, eps=1e-3):
    """v <- r + max_a discount * P_a v until max|dv| <= eps (solver.py:9-52)."""
    mdp = _model(p)
    v, _, _ = ops.value_iteration(mdp, reward, discount, eps, average=False, numpy_order=_np_order(mdp))
    return v[0].cpu().numpy()


def stochastic_value_iteration(p, reward, discount, eps=1e-3):
    """As value_iteration with the mean over actions instead of the max (solver.py:55-104)."""
    mdp = _model(p)
    v, _, _ = ops.value_iteration(mdp, reward, discount, eps, average=True, numpy_order=_np_order(mdp))
    return v[0].cpu().numpy()


def _uses_grid_transition(world):
    # the clipped-move successor of gridworld.py:54-122, not overridden by a subclass
    cls = type(world)
    names = ("state_index_transition", "state_index_to_point", "state_point_to_index_clipped",
             "state_point_to_index")
    return (hasattr(world, "size") and hasattr(world, "actions") and world.n_states == world.size ** 2
            and all(getattr(getattr(cls, n, None), "__qualname__", "") == f"GridWorld.{n}" for n in names))


def successor_table(world):
    """[S, A] int32 intended successors, world.state_index_transition(s, a)."""
    S, A = world.n_states, world.n_actions
    if _uses_grid_transition(world):
        size = world.size
        s = np.arange(S)
        x, y = s % size, s // size
        cols = []
        for a in range(A):
            dx, dy = world.actions[a]
            cx = np.clip(x + dx, 0, size - 1)
            cy = np.clip(y + dy, 0, size - 1)
            cols.append(cy * size + cx)
        return np.stack(cols, axis=1).astype(np.int32)
    return np.array([[world.state_index_transition(s, a) for a in range(A)] for s in range(S)],
                    dtype=np.int32)


def _device():
    from irlmx import require_device
    return require_device()


def optimal_policy_from_value(world, value):
    """Greedy action w.r.t. the intended successor's value (solver.py:107-124)."""
    dev = _device()
    succ = torch.as_tensor(successor_table(world), device=dev)
    v = torch.as_tensor(np.asarray(value, dtype=np.float64), device=dev)
    return ops.optimal_policy(succ, v)[0].cpu().numpy()


def optimal_policy(world, reward, discount, eps=1e-3):
    """value_iteration followed by optimal_policy_from_value (solver.py:127-152)."""
    value = value_iteration(world.p_transition, reward, discount, eps)
    return optimal_policy_from_value(world, value)


def stochastic_policy_from_value(world, value, w=lambda x: x):
    """Successor values weighted by ``w`` and normalised per state (solver.py:155-181)."""
    dev = _device()
    succ = torch.as_tensor(successor_table(world), device=dev)
    # w is arbitrary Python, applied per element exactly as the reference does
    # (to numpy float64 scalars); gathering and normalising run on the device
    wv = np.array([w(x) for x in np.asarray(value, dtype=np.float64)], dtype=np.float64)
    return ops.stochastic_policy(succ, torch.as_tensor(wv, device=dev))[0].cpu().numpy()
