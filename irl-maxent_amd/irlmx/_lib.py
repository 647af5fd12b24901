"""ctypes binding of libirlmx.so (the C ABI declared in include/irlmx.h).

torch is imported first on purpose: torch ships its own libamdhip64.so.7, and
loading it before libirlmx.so makes the dynamic loader resolve libirlmx's
HIP dependency to that same copy, so device pointers and streams created by
torch are valid inside the library (one HIP runtime per process).

There is no CPU fallback: if the library or a HIP device is missing, the ops
raise instead of computing anything elsewhere.
"""

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see above)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("IRLMX_LIB", os.path.join(_HERE, "libirlmx.so"))

LAYOUT_STENCIL5 = 1
LAYOUT_ELL = 2
LAYOUT_DENSE = 3

SUCCESS = 0
OK, NONFINITE, MAXITER = 0, 1, 2
OP_BACKWARD, OP_FORWARD, OP_SOFT_BACKWARD, OP_VALUE_ITERATION = 1, 2, 3, 4
PLAN_NO_RESCALE = 0x100
PROPS_KNOWN, PROP_COMPACT, PROP_ELL_SORTED = 0x40000000, 0x1, 0x2
EINVAL, EHIP, EWORKSPACE = -1, -2, -3
COUNTER_NAMES = ("cluster_launches", "grid_launches", "rerun_nonfinite", "rerun_not_resident", "rerun_timeout",
                 "sweep_calls")   # IRLMX_CTR_* order


class IrlmxError(RuntimeError):
    """A libirlmx call returned a negative status."""


class MDPStruct(ctypes.Structure):
    """Mirror of ``irlmx_mdp`` (include/irlmx.h)."""

    _fields_ = [
        ("layout", ctypes.c_int32),
        ("n_states", ctypes.c_int32),
        ("n_actions", ctypes.c_int32),
        ("width", ctypes.c_int32),
        ("height", ctypes.c_int32),
        ("k_row", ctypes.c_int32),
        ("k_col", ctypes.c_int32),
        ("batch", ctypes.c_int32),
        ("shared", ctypes.c_int32),
        ("props", ctypes.c_int32),
        ("row_val", ctypes.c_void_p),
        ("row_idx", ctypes.c_void_p),
        ("col_idx", ctypes.c_void_p),
        ("col_val", ctypes.c_void_p),
    ]


_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_D = ctypes.c_double
_SZ = ctypes.c_size_t
_MDP = ctypes.POINTER(MDPStruct)

# name -> (restype, argtypes); the exported-symbol list checked by the tests
SIGNATURES = {
    "irlmx_abi_version": (ctypes.c_int, []),
    "irlmx_last_error": (ctypes.c_char_p, []),
    "irlmx_counters": (ctypes.c_int, [_P, _I32]),
    "irlmx_workspace_bytes": (_SZ, [_MDP, _I32]),
    "irlmx_mdp_properties": (ctypes.c_int, [_MDP, _P, _P]),
    "irlmx_numpy_math": (ctypes.c_int, [ctypes.c_int32, _P, _P, ctypes.c_int64, _P]),
    "irlmx_device_checks_enabled": (ctypes.c_int, []),
    "irlmx_device_check_failures": (_I64, []),
    "irlmx_backward_maxent": (ctypes.c_int, [_MDP, _P, _P, _I32, _P, _P, _P, _SZ, _P]),
    "irlmx_backward_maxent_numpy_order": (ctypes.c_int, [_MDP, _P, _P, _P, _P, _P]),
    "irlmx_forward_svf_numpy_order": (ctypes.c_int, [_MDP, _P, _P, _P, _D, _I64, _P, _P, _P, _P]),
    "irlmx_forward_svf": (ctypes.c_int, [_MDP, _P, _P, _P, _D, _I64, _P, _P, _P, _P, _SZ, _P]),
    "irlmx_soft_backward": (ctypes.c_int, [_MDP, _P, _P, _D, _D, _I64, _P, _P, _P, _P, _P, _SZ, _P]),
    "irlmx_soft_backward_numpy_order": (ctypes.c_int, [_MDP, _P, _P, _D, _D, _I64, _P, _P, _P, _P, _P]),
    "irlmx_value_iteration_numpy_order": (ctypes.c_int, [_MDP, _P, _D, _D, _I32, _I64, _P, _P, _P, _P]),
    "irlmx_value_iteration": (ctypes.c_int, [_MDP, _P, _D, _D, _I32, _I64, _P, _P, _P, _P, _SZ, _P]),
    "irlmx_execution_plan": (ctypes.c_int, [_MDP, _I32, _P]),
    "irlmx_optimal_policy": (ctypes.c_int, [_P, _I32, _I32, _I32, _P, _P, _P]),
    "irlmx_stochastic_policy": (ctypes.c_int, [_P, _I32, _I32, _I32, _P, _P, _P]),
    "irlmx_build_icy_gridworld": (ctypes.c_int, [_I32, _P, _I32, _P, _P]),
    "irlmx_build_gridworld": (ctypes.c_int, [_I32, _I32, _P, _P]),
    "irlmx_dense_to_stencil": (ctypes.c_int, [_P, _I32, _I32, _I32, _P, _P, _P]),
    "irlmx_dense_to_rows": (ctypes.c_int, [_P, _I32, _I32, _P, _P, _P]),
    "irlmx_dense_ell_sizes": (ctypes.c_int, [_P, _I32, _I32, _P, _P, _P]),
    "irlmx_dense_to_ell": (ctypes.c_int, [_P, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _P]),
    "irlmx_dense_gemm": (ctypes.c_int, [_P, _P, _P, _I32, _I32, _I32, _P]),
    "irlmx_dense_gemm_variant": (ctypes.c_int, [_I32, _I32, _I32, _P]),
}

_lib = None
_load_error = None


def load():
    """Load libirlmx.so once; raise ImportError with the reason if it cannot be."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if _load_error is not None:
        raise ImportError(_load_error)
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as e:
        _load_error = (f"irlmx: cannot load {LIB_PATH} ({e}); build it with "
                       f"`python -c 'import __graft_entry__ as g; g.build()'`")
        raise ImportError(_load_error) from e
    variant = "IRLMX_LIB" in os.environ   # a diagnostic build may predate newer entry points
    for name, (res, args) in SIGNATURES.items():
        if variant and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.irlmx_abi_version() != 1:
        raise ImportError("irlmx: ABI version mismatch")
    _lib = lib
    return lib


def check(rc, what):
    if rc != SUCCESS:
        msg = load().irlmx_last_error().decode(errors="replace")
        raise IrlmxError(f"{what} failed ({rc}): {msg}")


def require_device(device=None):
    """The device every irlmx op runs on; raises when no HIP device exists."""
    load()
    if not torch.cuda.is_available():
        raise RuntimeError("irlmx: no HIP device available (the MI355X path has no CPU fallback)")
    if device is None:
        return torch.device("cuda", torch.cuda.current_device())
    device = torch.device(device)
    if device.type != "cuda":
        raise RuntimeError(f"irlmx: ops run on a HIP device, got {device}")
    return device


def stream_ptr(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)
