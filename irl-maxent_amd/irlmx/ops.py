"""Batched device operations of the MaxEnt-IRL inner loop (torch tensors in/out).

Every function runs on the HIP device through libirlmx.so; inputs are float64
(or uint8 masks) of shape [B, ...] and stay resident in HBM.  These are the
building blocks of the numpy drop-ins (``maxent``, ``solver``) and of the
batched IRL driver (``irlmx.batch``).
"""

import os

import numpy as np
import torch

from . import _lib
from .mdp import DeviceMDP

def _workspace(mdp, op):
    """Device workspace for one call, from torch's caching allocator.

    Allocated per call on the current stream: the allocator hands a freed block
    only to later work on the same stream (stream-ordered), so concurrent calls
    from other host threads or on other streams never share a workspace that an
    in-flight kernel still uses -- the stream / thread safety include/irlmx.h
    states for the C ABI."""
    lib = _lib.load()
    n = int(lib.irlmx_workspace_bytes(mdp.struct(), op))
    return torch.empty(max(n, 256), dtype=torch.uint8, device=mdp.device), n


PLAN_FIELDS = ("shape", "R", "G", "C", "per_launch", "spt", "layout", "threads", "launches", "lds_bytes")
SHAPES = {0: "fused", 1: "cluster", 2: "sweep", 3: "dense", 4: "dense-gemm", 5: "grid", 6: "dense-grid"}
_OPS = {"backward": _lib.OP_BACKWARD, "forward": _lib.OP_FORWARD, "soft_backward": _lib.OP_SOFT_BACKWARD,
        "value_iteration": _lib.OP_VALUE_ITERATION}


def execution_plan(mdp, op, rescale=True):
    """The kernel plan a call of ``op`` ("backward", "forward", "soft_backward",
    "value_iteration") on ``mdp`` runs on the current device (irlmx_execution_plan):
    shape, tile rows R, ghost rows G, tiles per instance C, instances per launch,
    states per lane, in-tile layout, threads, sequential launches, LDS bytes.
    ``rescale=False``: the plan of ``backward_maxent(..., rescale=False)``."""
    import ctypes
    lib = _lib.load()
    buf = (ctypes.c_int64 * len(PLAN_FIELDS))()
    code = _OPS[op] | (0 if rescale or op != "backward" else _lib.PLAN_NO_RESCALE)
    _lib.check(lib.irlmx_execution_plan(mdp.struct(), code, buf), "execution_plan")
    plan = dict(zip(PLAN_FIELDS, [int(v) for v in buf]))
    plan["shape"] = SHAPES[plan["shape"]]
    return plan


def counters():
    """Process-wide event counters of the library (irlmx_counters): persistent
    launches and per-sweep reruns, by name (``_lib.COUNTER_NAMES``)."""
    import ctypes
    lib = _lib.load()
    buf = (ctypes.c_int64 * len(_lib.COUNTER_NAMES))()
    n = lib.irlmx_counters(buf, len(_lib.COUNTER_NAMES))
    assert n == len(_lib.COUNTER_NAMES), n
    return dict(zip(_lib.COUNTER_NAMES, [int(v) for v in buf]))


def device_check_failures():
    """Bits of the in-kernel bounds checks that failed since the last call
    (irlmx_device_check_failures: 1 index, 2 granule, 4 tile); always 0 unless
    the library is the IRLMX_DEVICE_CHECKS build (libirlmx_checks.so)."""
    v = int(_lib.load().irlmx_device_check_failures())
    if v < 0:
        raise RuntimeError("irlmx_device_check_failures: HIP error")
    return v


def _f64(x, mdp, shape):
    t = torch.as_tensor(x, dtype=torch.float64, device=mdp.device)
    return t.reshape(shape).contiguous()


def terminal_mask(terminal, n_states, batch=1, device=None):
    """uint8 [B, S] mask with the reference's indexing semantics (maxent.py:99, 147).

    ``terminal`` is indexed into a numpy vector exactly as the reference indexes
    with it, so negative indices, duplicates and invalid index types behave (or
    raise) the same way.
    """
    m = np.zeros(n_states, dtype=np.uint8)
    m[terminal] = 1
    return torch.as_tensor(np.tile(m, (batch, 1)), device=device)


def backward_maxent(mdp, reward, terminal, rescale=True):
    """Local action probabilities [B, S, A] (maxent.py:119-159)."""
    lib = _lib.load()
    B, S, A = mdp.batch, mdp.n_states, mdp.n_actions
    r = _f64(reward, mdp, (B, S))
    term = terminal.to(device=mdp.device, dtype=torch.uint8).reshape(B, S).contiguous()
    pi = torch.empty((B, S, A), dtype=torch.float64, device=mdp.device)
    status = torch.empty(B, dtype=torch.int32, device=mdp.device)
    ws, n = _workspace(mdp, _lib.OP_BACKWARD)
    _lib.check(lib.irlmx_backward_maxent(mdp.struct(), _lib.ptr(r), _lib.ptr(term), 1 if rescale else 0,
                                         _lib.ptr(pi), _lib.ptr(status), _lib.ptr(ws), n,
                                         _lib.stream_ptr(mdp.device)), "backward_maxent")
    return pi


def numpy_order_supported(mdp, op="backward"):
    """Whether the numpy-order kernels cover this model (S <= 4096, S % 4 in
    {0, 1}; the forward's ELL column form at most 32 slots)."""
    S = mdp.n_states
    ok = S <= 4096 and S % 4 in (0, 1)
    if op == "forward" and mdp.layout == _lib.LAYOUT_ELL:
        ok = ok and mdp.k_col <= 32
    return ok


# Default numpy-order scope of the drop-ins per op: (states on STENCIL5 / ELL
# models, states on DENSE tables).  The kernels themselves cover 4096 states.
NUMPY_ORDER_CAPS = {"backward": (1024, 64), "forward": (1024, 64),
                    "soft_backward": (4096, 64), "value_iteration": (4096, 4096)}
_CAP_ENV = {"backward": "BWD", "forward": "FWD", "soft_backward": "SOFT", "value_iteration": "VI"}


def numpy_order_cap(mdp, op="backward"):
    """The largest state count at which the drop-ins run ``op`` in numpy's order
    on this model's layout (NUMPY_ORDER_CAPS; environment overrides: see
    numpy_order_default)."""
    sparse_cap, dense_cap = NUMPY_ORDER_CAPS[op]
    cap = int(os.environ.get("IRLMX_NUMPY_ORDER_MAX", sparse_cap))
    cap = int(os.environ.get(f"IRLMX_NUMPY_ORDER_{_CAP_ENV[op]}_MAX", cap))
    if mdp.layout == _lib.LAYOUT_DENSE:
        cap = min(cap, int(os.environ.get("IRLMX_NUMPY_ORDER_DENSE_MAX", dense_cap)))
    return cap


def numpy_order_default(mdp, op="backward"):
    """Whether the drop-ins (maxent.py, solver.py) run ``op`` ("backward",
    "forward", "soft_backward", "value_iteration") in numpy's order: one
    instance, a model the numpy-order kernels cover, and at most
    numpy_order_cap(mdp, op) states.

    Caps per op (NUMPY_ORDER_CAPS): value iteration and soft VI run in numpy's
    order on every model the kernels cover (4096 states; soft VI 64 on a DENSE
    table), so solver.value_iteration / optimal_policy and
    local_causal_action_probabilities reproduce the reference's values and argmax
    at config 2's 64x64 (tests/golden/c2_64.npz).  The backward and the forward
    stop at 1024 (64 on DENSE): beyond, their one-workgroup kernels re-read every
    entry each of thousands of sweeps -- measured on one MI355X
    (tools/diag/np_bwd_cost.py), the backward takes 31-435x the tiled shapes' time
    at 33x33-64x64 (1.26 s vs 2.9 ms at 64x64) and 132x / 1,650x on dense tables of
    256 / 1024 states; soft VI costs 4-16x on grids (milliseconds) but 75-950x on
    dense tables, value iteration (tens of sweeps) stays in milliseconds to a
    fraction of a second.  Above the caps the drop-ins take the tiled shapes
    (within 1e-9 of the oracle; argmax ties may fall differently).

    Environment: IRLMX_NUMPY_ORDER=0 turns numpy's order off;
    IRLMX_NUMPY_ORDER_MAX sets every op's grid cap, IRLMX_NUMPY_ORDER_{BWD,FWD,
    SOFT,VI}_MAX one op's, IRLMX_NUMPY_ORDER_DENSE_MAX the DENSE cap."""
    if mdp.batch != 1 or not numpy_order_supported(mdp, op) or os.environ.get("IRLMX_NUMPY_ORDER", "1") == "0":
        return False
    return mdp.n_states <= numpy_order_cap(mdp, op)


def backward_maxent_numpy_order(mdp, exp_reward, terminal):
    """Local action probabilities [B, S, A] (maxent.py:119-159) in numpy's own
    floating-point order (irlmx_backward_maxent_numpy_order): bit-identical to
    the reference's on a Haswell-family OpenBLAS host, NaN where it overflows.
    ``exp_reward`` is np.exp(reward) as the reference computes it (maxent.py:142)."""
    lib = _lib.load()
    B, S, A = mdp.batch, mdp.n_states, mdp.n_actions
    er = _f64(exp_reward, mdp, (B, S))
    term = terminal.to(device=mdp.device, dtype=torch.uint8).reshape(B, S).contiguous()
    pi = torch.empty((B, S, A), dtype=torch.float64, device=mdp.device)
    status = torch.empty(B, dtype=torch.int32, device=mdp.device)
    _lib.check(lib.irlmx_backward_maxent_numpy_order(mdp.struct(), _lib.ptr(er), _lib.ptr(term), _lib.ptr(pi),
                                                     _lib.ptr(status), _lib.stream_ptr(mdp.device)),
               "backward_maxent_numpy_order")
    return pi


def forward_svf(mdp, p_initial, terminal, p_action, eps=1e-5, max_iter=0, numpy_order=False):
    """Expected state-visitation frequencies (maxent.py:63-114).

    Returns ``(svf [B, S], iterations [B] int64, status [B] int32)``.
    ``numpy_order``: numpy's summation order (irlmx_forward_svf_numpy_order):
    SVF and sweep count bit-identical to the reference on a Haswell-family host.
    """
    lib = _lib.load()
    B, S, A = mdp.batch, mdp.n_states, mdp.n_actions
    p0 = _f64(p_initial, mdp, (B, S))
    pi = _f64(p_action, mdp, (B, S, A))
    term = terminal.to(device=mdp.device, dtype=torch.uint8).reshape(B, S).contiguous()
    svf = torch.empty((B, S), dtype=torch.float64, device=mdp.device)
    iters = torch.empty(B, dtype=torch.int64, device=mdp.device)
    status = torch.empty(B, dtype=torch.int32, device=mdp.device)
    if numpy_order:
        _lib.check(lib.irlmx_forward_svf_numpy_order(mdp.struct(), _lib.ptr(p0), _lib.ptr(term), _lib.ptr(pi),
                                                     float(eps), int(max_iter), _lib.ptr(svf), _lib.ptr(iters),
                                                     _lib.ptr(status), _lib.stream_ptr(mdp.device)),
                   "forward_svf_numpy_order")
        return svf, iters, status
    ws, n = _workspace(mdp, _lib.OP_FORWARD)
    _lib.check(lib.irlmx_forward_svf(mdp.struct(), _lib.ptr(p0), _lib.ptr(term), _lib.ptr(pi), float(eps),
                                     int(max_iter), _lib.ptr(svf), _lib.ptr(iters), _lib.ptr(status),
                                     _lib.ptr(ws), n, _lib.stream_ptr(mdp.device)), "forward_svf")
    return svf, iters, status


def soft_backward(mdp, reward, terminal_reward, discount, eps=1e-5, max_iter=0, numpy_order=False):
    """MaxCausalEnt soft value iteration (maxent.py:279-341).

    Returns ``(p_action [B, S, A], value [B, S], iterations [B], status [B])``.
    ``numpy_order``: every P_a . v summed in numpy's order
    (irlmx_soft_backward_numpy_order; numpy_order_supported(mdp) models only).
    """
    lib = _lib.load()
    B, S, A = mdp.batch, mdp.n_states, mdp.n_actions
    r = _f64(reward, mdp, (B, S))
    phi = _f64(terminal_reward, mdp, (B, S))
    pi = torch.empty((B, S, A), dtype=torch.float64, device=mdp.device)
    v = torch.empty((B, S), dtype=torch.float64, device=mdp.device)
    iters = torch.empty(B, dtype=torch.int64, device=mdp.device)
    status = torch.empty(B, dtype=torch.int32, device=mdp.device)
    if numpy_order:
        _lib.check(lib.irlmx_soft_backward_numpy_order(mdp.struct(), _lib.ptr(r), _lib.ptr(phi), float(discount),
                                                       float(eps), int(max_iter), _lib.ptr(pi), _lib.ptr(v),
                                                       _lib.ptr(iters), _lib.ptr(status), _lib.stream_ptr(mdp.device)),
                   "soft_backward_numpy_order")
        return pi, v, iters, status
    ws, n = _workspace(mdp, _lib.OP_SOFT_BACKWARD)
    _lib.check(lib.irlmx_soft_backward(mdp.struct(), _lib.ptr(r), _lib.ptr(phi), float(discount), float(eps),
                                       int(max_iter), _lib.ptr(pi), _lib.ptr(v), _lib.ptr(iters),
                                       _lib.ptr(status), _lib.ptr(ws), n, _lib.stream_ptr(mdp.device)),
               "soft_backward")
    return pi, v, iters, status


def value_iteration(mdp, reward, discount, eps=1e-3, average=False, max_iter=0, numpy_order=False):
    """Hard-max (solver.py:9-52) or action-average (solver.py:55-104) value iteration.

    Returns ``(value [B, S], iterations [B], status [B])``.  ``numpy_order``:
    numpy's summation order (irlmx_value_iteration_numpy_order), values
    bit-identical to the reference's on a Haswell-family OpenBLAS host.
    """
    lib = _lib.load()
    B, S = mdp.batch, mdp.n_states
    r = _f64(reward, mdp, (B, S))
    v = torch.empty((B, S), dtype=torch.float64, device=mdp.device)
    iters = torch.empty(B, dtype=torch.int64, device=mdp.device)
    status = torch.empty(B, dtype=torch.int32, device=mdp.device)
    if numpy_order:
        _lib.check(lib.irlmx_value_iteration_numpy_order(mdp.struct(), _lib.ptr(r), float(discount), float(eps),
                                                         1 if average else 0, int(max_iter), _lib.ptr(v),
                                                         _lib.ptr(iters), _lib.ptr(status),
                                                         _lib.stream_ptr(mdp.device)), "value_iteration_numpy_order")
        return v, iters, status
    ws, n = _workspace(mdp, _lib.OP_VALUE_ITERATION)
    _lib.check(lib.irlmx_value_iteration(mdp.struct(), _lib.ptr(r), float(discount), float(eps),
                                         1 if average else 0, int(max_iter), _lib.ptr(v), _lib.ptr(iters),
                                         _lib.ptr(status), _lib.ptr(ws), n, _lib.stream_ptr(mdp.device)),
               "value_iteration")
    return v, iters, status


def dense_gemm(m, z):
    """``z @ m.T`` on the fp64 matrix cores (irlmx_dense_gemm): m [R, S], z [B, S]
    float64 device tensors -> [B, R].  The batched P . [v_1 .. v_B] contraction
    of the DENSE layout's shared-table sweeps."""
    lib = _lib.load()
    m = m.to(dtype=torch.float64).contiguous()
    z = z.to(dtype=torch.float64, device=m.device).contiguous()
    (R, S), (B, S2) = m.shape, z.shape
    if S2 != S:
        raise ValueError(f"dense_gemm: m is {tuple(m.shape)}, z is {tuple(z.shape)}")
    c = torch.empty((B, R), dtype=torch.float64, device=m.device)
    _lib.check(lib.irlmx_dense_gemm(_lib.ptr(m), _lib.ptr(z), _lib.ptr(c), R, S, B, _lib.stream_ptr(m.device)),
               "dense_gemm")
    return c


def dense_gemm_variant(rows, n, batch):
    """(row tiles, instance tiles, waves, 16-byte loads) of the MFMA kernel a
    dense_gemm of these sizes launches."""
    import ctypes
    lib = _lib.load()
    v = (ctypes.c_int32 * 4)()
    _lib.check(lib.irlmx_dense_gemm_variant(rows, n, batch, v), "dense_gemm_variant")
    return tuple(int(x) for x in v)


def optimal_policy(successor, value):
    """argmax_a value[successor[s, a]] per state, first index on ties (solver.py:107-124)."""
    lib = _lib.load()
    succ = successor.to(dtype=torch.int32).contiguous()
    S, A = succ.shape
    value = value.to(dtype=torch.float64).reshape(-1, S).contiguous()
    B = value.shape[0]
    out = torch.empty((B, S), dtype=torch.int64, device=value.device)
    _lib.check(lib.irlmx_optimal_policy(_lib.ptr(succ), S, A, B, _lib.ptr(value), _lib.ptr(out),
                                        _lib.stream_ptr(value.device)), "optimal_policy")
    return out


def stochastic_policy(successor, weighted_value):
    """w(value)[successor] normalised per state (solver.py:155-181)."""
    lib = _lib.load()
    succ = successor.to(dtype=torch.int32).contiguous()
    S, A = succ.shape
    wv = weighted_value.to(dtype=torch.float64).reshape(-1, S).contiguous()
    B = wv.shape[0]
    out = torch.empty((B, S, A), dtype=torch.float64, device=wv.device)
    _lib.check(lib.irlmx_stochastic_policy(_lib.ptr(succ), S, A, B, _lib.ptr(wv), _lib.ptr(out),
                                           _lib.stream_ptr(wv.device)), "stochastic_policy")
    return out


__all__ = ["DeviceMDP", "execution_plan", "numpy_order_default", "counters", "terminal_mask", "backward_maxent", "forward_svf", "soft_backward",
           "value_iteration", "dense_gemm", "dense_gemm_variant", "optimal_policy", "stochastic_policy"]
