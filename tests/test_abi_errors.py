"""Failure paths of the C ABI (include/irlmx.h return codes), through ctypes.

Every entry point rejects bad arguments before it enqueues any work: a
negative IRLMX_E* code plus a message in irlmx_last_error().  The calls below
all fail in that argument check, so the non-NULL array pointers they pass are
never dereferenced (host addresses stand in for device buffers) and no GPU is
needed; the same checks hold on a GPU box.  The paths that need a device
(co-residency rejection, exchange timeout) are in tests/test_gpu_errors.py.
"""

import ctypes

import pytest

EINVAL, EHIP, EWORKSPACE = -1, -2, -3


@pytest.fixture(scope="module")
def lib():
    import __graft_entry__ as g
    g.build()
    from irlmx import _lib
    return _lib.load()


_keep = []


def fake():
    """A non-NULL address that the argument checks never dereference."""
    b = ctypes.create_string_buffer(64)
    _keep.append(b)
    return ctypes.cast(b, ctypes.c_void_p)


NULL = ctypes.c_void_p(0)


def model(layout=1, S=25, A=4, W=5, H=5, k_row=5, k_col=5, B=1, shared=1, row_val=True, row_idx=False,
          col_idx=False, col_val=False):
    from irlmx import _lib
    m = _lib.MDPStruct()
    m.layout, m.n_states, m.n_actions, m.width, m.height = layout, S, A, W, H
    m.k_row, m.k_col, m.batch, m.shared = k_row, k_col, B, shared
    for name, on in (("row_val", row_val), ("row_idx", row_idx), ("col_idx", col_idx), ("col_val", col_val)):
        setattr(m, name, fake().value if on else None)
    return m


def err(lib):
    return lib.irlmx_last_error().decode()


# entry points taking a model: name -> (op code, call(lib, mdp_ptr, args dict) -> rc, required array args)
def _bwd(lib, m, a):
    return lib.irlmx_backward_maxent(m, a["reward"], a["terminal"], 1, a["p_action"], a["status"], a["ws"], a["n"],
                                     NULL)


def _fwd(lib, m, a):
    return lib.irlmx_forward_svf(m, a["p_initial"], a["terminal"], a["p_action"], 1e-5, 0, a["svf"], a["iterations"],
                                 a["status"], a["ws"], a["n"], NULL)


def _soft(lib, m, a):
    return lib.irlmx_soft_backward(m, a["reward"], a["terminal_reward"], 0.7, 1e-5, 0, a["p_action"], a["value"],
                                   a["iterations"], a["status"], a["ws"], a["n"], NULL)


def _vi(lib, m, a):
    return lib.irlmx_value_iteration(m, a["reward"], 0.9, 1e-3, 0, 0, a["value"], a["iterations"], a["status"],
                                     a["ws"], a["n"], NULL)


def _bwd_np(lib, m, a):
    return lib.irlmx_backward_maxent_numpy_order(m, a["exp_reward"], a["terminal"], a["p_action"], a["status"], NULL)


def _fwd_np(lib, m, a):
    return lib.irlmx_forward_svf_numpy_order(m, a["p_initial"], a["terminal"], a["p_action"], 1e-5, 0, a["svf"],
                                             a["iterations"], a["status"], NULL)


def _soft_np(lib, m, a):
    return lib.irlmx_soft_backward_numpy_order(m, a["reward"], a["terminal_reward"], 0.7, 1e-5, 0, a["p_action"],
                                               a["value"], a["iterations"], a["status"], NULL)


def _vi_np(lib, m, a):
    return lib.irlmx_value_iteration_numpy_order(m, a["reward"], 0.9, 1e-3, 0, 0, a["value"], a["iterations"],
                                                 a["status"], NULL)


ENTRY = {
    "backward_maxent": (1, _bwd, ("reward", "terminal", "p_action", "status")),
    "backward_maxent_numpy_order": (1, _bwd_np, ("exp_reward", "terminal", "p_action", "status")),
    "forward_svf": (2, _fwd, ("p_initial", "terminal", "p_action", "svf", "iterations", "status")),
    "soft_backward": (3, _soft, ("reward", "terminal_reward", "p_action", "iterations", "status")),
    "value_iteration": (4, _vi, ("reward", "value", "iterations", "status")),
    "forward_svf_numpy_order": (2, _fwd_np, ("p_initial", "terminal", "p_action", "svf", "iterations", "status")),
    "soft_backward_numpy_order": (3, _soft_np, ("reward", "terminal_reward", "p_action", "iterations", "status")),
    "value_iteration_numpy_order": (4, _vi_np, ("reward", "value", "iterations", "status")),
}
NO_WORKSPACE = {"backward_maxent_numpy_order", "forward_svf_numpy_order", "soft_backward_numpy_order",
                "value_iteration_numpy_order"}
ARGS = ("reward", "terminal", "p_action", "status", "p_initial", "svf", "iterations", "terminal_reward", "value",
        "exp_reward")


def args_for(lib, m, op, **over):
    a = {k: fake() for k in ARGS}
    n = int(lib.irlmx_workspace_bytes(ctypes.byref(m), op))
    a["ws"], a["n"] = fake(), n
    a.update(over)
    return a


BAD_MODELS = [
    ("S=0", dict(S=0), "bad sizes S=0"),
    ("A=0", dict(A=0), "bad sizes"),
    ("B=0", dict(B=0), "bad sizes"),
    ("B<0", dict(B=-3), "bad sizes"),
    ("A=9", dict(A=9), "n_actions=9 exceeds 8"),
    ("row_val NULL", dict(row_val=False), "row_val is NULL"),
    ("grid != S", dict(W=4), "stencil grid 4x5 != 25 states"),
    ("negative grid", dict(W=-5, H=-5), "stencil grid -5x-5"),
    ("unknown layout", dict(layout=7), "unknown layout 7"),
    ("ELL row_idx NULL", dict(layout=2, k_row=3), "ELL row form missing"),
    ("ELL k_row 0", dict(layout=2, k_row=0, row_idx=True), "ELL row form missing"),
    ("ELL k_row > S", dict(layout=2, k_row=26, row_idx=True), "ELL k_row=26 out of range"),
    ("DENSE col_val NULL", dict(layout=3, k_row=25, k_col=25), "col_val) missing"),
    ("DENSE too large", dict(layout=3, S=1 << 20, k_row=1 << 20, k_col=1 << 20, col_val=True), "DENSE table too large"),
]


@pytest.mark.parametrize("fn", sorted(ENTRY))
@pytest.mark.parametrize("case,kw,msg", BAD_MODELS, ids=[c[0] for c in BAD_MODELS])
def test_bad_model_einval(lib, fn, case, kw, msg):
    op, call, _ = ENTRY[fn]
    good = model()
    a = args_for(lib, good, op)
    m = model(**kw)
    assert call(lib, ctypes.byref(m), a) == EINVAL
    assert msg in err(lib), (fn, case, err(lib))
    # the model query functions: no workspace for an invalid model, and the same error for the plan
    assert lib.irlmx_workspace_bytes(ctypes.byref(m), op) == 0
    plan = (ctypes.c_int64 * 10)()
    assert lib.irlmx_execution_plan(ctypes.byref(m), op, plan) == EINVAL and msg in err(lib)


@pytest.mark.parametrize("fn", sorted(ENTRY))
def test_null_model_einval(lib, fn):
    op, call, _ = ENTRY[fn]
    a = args_for(lib, model(), op)
    assert call(lib, None, a) == EINVAL and err(lib) == "mdp is NULL"


@pytest.mark.parametrize("fn", sorted(ENTRY))
def test_null_required_array_einval(lib, fn):
    op, call, required = ENTRY[fn]
    m = model()
    for name in required:
        a = args_for(lib, m, op, **{name: NULL})
        assert call(lib, ctypes.byref(m), a) == EINVAL, (fn, name)
        assert err(lib) == f"{fn}: {name} is NULL", (fn, name, err(lib))


def test_optional_arrays_accepted_as_null(lib):
    """soft_backward's value output may be NULL (irlmx.h); the call then gets as
    far as the workspace check (here: too small, so nothing is enqueued)."""
    m = model()
    a = args_for(lib, m, 3, value=NULL, n=0, ws=NULL)
    assert _soft(lib, ctypes.byref(m), a) == EWORKSPACE


@pytest.mark.parametrize("fn", sorted(set(ENTRY) - NO_WORKSPACE))
@pytest.mark.parametrize("layout", ["stencil", "ell", "dense"])
def test_workspace_too_small(lib, fn, layout):
    op, call, _ = ENTRY[fn]
    kw = {"stencil": {}, "ell": dict(layout=2, k_row=3, k_col=3, row_idx=True, col_idx=True, col_val=True),
          "dense": dict(layout=3, k_row=25, k_col=25, col_val=True)}[layout]
    m = model(B=4, shared=0, **kw)
    need = int(lib.irlmx_workspace_bytes(ctypes.byref(m), op))
    assert need > 0
    for got, ws in ((0, fake()), (need - 1, fake()), (need, NULL)):
        a = args_for(lib, m, op, n=got, ws=ws)
        assert call(lib, ctypes.byref(m), a) == EWORKSPACE, (fn, layout, got)
        assert err(lib) == f"workspace too small: need {need} bytes, got {got}", err(lib)


def test_forward_ell_column_form(lib):
    m = model(layout=2, k_row=3, k_col=3, row_idx=True)      # column form missing
    a = args_for(lib, model(), 2)
    assert _fwd(lib, ctypes.byref(m), a) == EINVAL and err(lib) == "ELL column form missing"
    m = model(layout=2, k_row=3, k_col=40, row_idx=True, col_idx=True, col_val=True)
    assert _fwd(lib, ctypes.byref(m), a) == EINVAL and "ELL k_col=40 out of range" in err(lib)


def test_execution_plan_arguments(lib):
    m = model()
    assert lib.irlmx_execution_plan(ctypes.byref(m), 1, None) == EINVAL and err(lib) == "plan is NULL"
    plan = (ctypes.c_int64 * 10)()
    for op in (0, 5, -1):
        assert lib.irlmx_execution_plan(ctypes.byref(m), op, plan) == EINVAL and err(lib) == f"unknown op {op}"
    assert lib.irlmx_execution_plan(ctypes.byref(m), 2 | 0x100, plan) == EINVAL
    assert "NO_RESCALE applies to IRLMX_OP_BACKWARD only" in err(lib)


def test_mdp_properties_arguments(lib):
    """irlmx_mdp_properties validates before it touches the device: a NULL model,
    a NULL result pointer and every bad model are IRLMX_EINVAL."""
    assert lib.irlmx_mdp_properties(None, fake(), NULL) == EINVAL and err(lib) == "mdp is NULL"
    m = model()
    assert lib.irlmx_mdp_properties(ctypes.byref(m), None, NULL) == EINVAL
    assert err(lib) == "mdp_properties: props is NULL"
    for case, kw, msg in BAD_MODELS:
        bad = model(**kw)
        assert lib.irlmx_mdp_properties(ctypes.byref(bad), fake(), NULL) == EINVAL, case
        assert msg in err(lib), (case, err(lib))


def test_world_builders_and_converters(lib):
    f = fake
    cases = [
        (lambda: lib.irlmx_build_icy_gridworld(0, f(), 1, f(), NULL), "build_icy_gridworld: bad arguments (size=0"),
        (lambda: lib.irlmx_build_icy_gridworld(50000, f(), 1, f(), NULL), "size=50000"),
        (lambda: lib.irlmx_build_icy_gridworld(5, NULL, 1, f(), NULL), "p_slip NULL"),
        (lambda: lib.irlmx_build_icy_gridworld(5, f(), 0, f(), NULL), "batch=0"),
        (lambda: lib.irlmx_build_icy_gridworld(5, f(), 1, NULL, NULL), "row_val NULL"),
        (lambda: lib.irlmx_build_gridworld(-1, 1, f(), NULL), "build_gridworld: bad arguments (size=-1"),
        (lambda: lib.irlmx_build_gridworld(5, 1, NULL, NULL), "row_val NULL"),
        (lambda: lib.irlmx_dense_to_stencil(f(), 0, 5, 4, f(), f(), NULL), "dense_to_stencil: bad arguments (width=0"),
        (lambda: lib.irlmx_dense_to_stencil(f(), 5, 5, 4, f(), NULL, NULL), "off_stencil NULL"),
        (lambda: lib.irlmx_dense_to_stencil(NULL, 5, 5, 4, f(), f(), NULL), "dense NULL"),
        (lambda: lib.irlmx_dense_to_rows(f(), 0, 4, f(), f(), NULL), "dense_to_rows: bad arguments"),
        (lambda: lib.irlmx_dense_to_rows(f(), 25, 9, f(), f(), NULL), "dense_to_rows: bad arguments"),
        (lambda: lib.irlmx_dense_ell_sizes(f(), 25, 0, f(), f(), NULL), "dense_ell_sizes: bad arguments"),
        (lambda: lib.irlmx_dense_ell_sizes(f(), 25, 4, NULL, f(), NULL), "k_out NULL"),
        (lambda: lib.irlmx_dense_to_ell(f(), 25, 4, 0, 3, f(), f(), f(), f(), NULL), "k_row=0"),
        (lambda: lib.irlmx_dense_to_ell(f(), 25, 4, 26, 3, f(), f(), f(), f(), NULL), "k_row=26"),
        (lambda: lib.irlmx_dense_to_ell(f(), 25, 4, 3, 3, f(), NULL, f(), f(), NULL), "every array non-NULL"),
        (lambda: lib.irlmx_optimal_policy(f(), 25, 4, 0, f(), f(), NULL), "optimal_policy: bad arguments"),
        (lambda: lib.irlmx_optimal_policy(f(), 25, 4, 1, NULL, f(), NULL), "value NULL"),
        (lambda: lib.irlmx_stochastic_policy(f(), 0, 4, 1, f(), f(), NULL), "stochastic_policy: bad arguments"),
        (lambda: lib.irlmx_stochastic_policy(NULL, 25, 4, 1, f(), f(), NULL), "successor NULL"),
    ]
    for call, msg in cases:
        assert call() == EINVAL, msg
        assert msg in err(lib), (msg, err(lib))


def test_error_text_is_per_thread(lib):
    """irlmx_last_error() is thread-local (irlmx.h): a failure on one thread does
    not overwrite the message another thread reads."""
    import threading
    m = model(S=0)
    a = args_for(lib, model(), 1)
    assert _bwd(lib, ctypes.byref(m), a) == EINVAL
    mine = err(lib)
    seen = {}

    def other():
        m2 = model(A=9)
        _bwd(lib, ctypes.byref(m2), args_for(lib, model(), 1))
        seen["msg"] = err(lib)

    t = threading.Thread(target=other)
    t.start()
    t.join()
    assert "exceeds 8" in seen["msg"] and err(lib) == mine


def test_counters_and_python_errors(lib):
    from irlmx import _lib, ops
    assert lib.irlmx_counters(None, 0) == len(_lib.COUNTER_NAMES)
    c = ops.counters()
    assert set(c) == set(_lib.COUNTER_NAMES) and all(v >= 0 for v in c.values())
    m = model(S=0)
    rc = _bwd(lib, ctypes.byref(m), args_for(lib, model(), 1))
    with pytest.raises(_lib.IrlmxError, match=r"backward_maxent failed \(-1\): bad sizes S=0"):
        _lib.check(rc, "backward_maxent")


@pytest.mark.parametrize("S,W,H", [(6, 2, 3), (7, 7, 1), (4097, 4097, 1), (65 * 65, 65, 65)])
def test_numpy_order_sizes_einval(lib, S, W, H):
    """numpy's order is restated for S <= 4096 with S % 4 in {0, 1} only
    (oracle/blas_order.c): other sizes are rejected, not approximated."""
    m = model(S=S, W=W, H=H)
    for call, op in ((_bwd_np, 1), (_fwd_np, 2), (_soft_np, 3), (_vi_np, 4)):
        a = args_for(lib, model(), op)
        assert call(lib, ctypes.byref(m), a) == EINVAL
        assert "numpy's order is restated for S <= 4096" in err(lib), err(lib)
