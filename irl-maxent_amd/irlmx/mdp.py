"""Transition models resident in HBM.

The reference hands the solvers a dense float64 ``p_transition[from, to,
action]`` (gridworld.py:124-142) and re-slices it per call (maxent.py:98-102,
143, 320; solver.py:37).  ``DeviceMDP`` holds the same model once, compactly:

* ``STENCIL5`` -- every nonzero of P lies on the 5-point stencil of a
  width x height grid (all reference gridworlds).  ``row_val[b][a][k][s]`` is
  ``P[s, nbr_k(s), a]`` for k = self, +x, -x, +y, -y: 5*A float64 per state
  (160 B at A = 4) instead of S*A*8 B per state dense.
* ``ELL`` -- any other sparsity: per state the union of targets over actions
  (row form, ``row_idx``/``row_val``) and, for the forward pass, the union of
  sources (column form, ``col_idx``/``col_val``).
* ``DENSE`` -- rows mostly nonzero (ELL would gather ~S slots per state): the
  per-action matrices ``row_val[b][a][s][t] = P[s, t, a]`` (the reference's
  slices ``P[:, :, a]``) and their action sum ``col_val[b][s][t]``, streamed
  row by row (dense.hip).

Instances: a model holds B tables, or one table shared by B instances
(``shared=True``), e.g. one world with B reward vectors.
"""

import ctypes
import math
import weakref

import numpy as np
import torch

from . import _lib


def _is_square(n):
    r = math.isqrt(n)
    return r if r * r == n else 0


class DeviceMDP:
    def __init__(self, layout, n_states, n_actions, batch, shared, row_val, row_idx=None,
                 col_idx=None, col_val=None, width=0, height=0, k_row=5, k_col=5, device=None):
        self.layout = layout
        self.n_states = int(n_states)
        self.n_actions = int(n_actions)
        self.batch = int(batch)
        self.shared = bool(shared)
        self.row_val = row_val
        self.row_idx = row_idx
        self.col_idx = col_idx
        self.col_val = col_val
        self.width = int(width)
        self.height = int(height)
        self.k_row = int(k_row)
        self.k_col = int(k_col)
        self.device = device if device is not None else row_val.device
        self._struct = None

    # -- construction ------------------------------------------------------

    @classmethod
    def icy_gridworld(cls, size, p_slip=0.2, device=None):
        """IcyGridWorld(size, p_slip) tables built on the device (gridworld.py:177-248).

        ``p_slip`` may be a sequence: one table per value (batch = len(p_slip)).
        """
        device = _lib.require_device(device)
        lib = _lib.load()
        slips = np.atleast_1d(np.asarray(p_slip, dtype=np.float64))
        B, S = len(slips), size * size
        d_slip = torch.as_tensor(slips, device=device)
        row_val = torch.empty((B, 4, 5, S), dtype=torch.float64, device=device)
        _lib.check(lib.irlmx_build_icy_gridworld(size, _lib.ptr(d_slip), B, _lib.ptr(row_val),
                                                 _lib.stream_ptr(device)), "build_icy_gridworld")
        return cls(_lib.LAYOUT_STENCIL5, S, 4, B, False, row_val, width=size, height=size, device=device)

    @classmethod
    def gridworld(cls, size, batch=1, device=None):
        """Deterministic GridWorld(size) tables (gridworld.py:23-171)."""
        device = _lib.require_device(device)
        lib = _lib.load()
        S = size * size
        row_val = torch.empty((batch, 4, 5, S), dtype=torch.float64, device=device)
        _lib.check(lib.irlmx_build_gridworld(size, batch, _lib.ptr(row_val), _lib.stream_ptr(device)),
                   "build_gridworld")
        return cls(_lib.LAYOUT_STENCIL5, S, 4, batch, False, row_val, width=size, height=size, device=device)

    def with_stay(self):
        """The same STENCIL5 tables with a fifth action "stay" (P[s, s, 4] = 1):
        BASELINE config 2's |A| = 5 variant of the gridworlds (SURVEY.md 8(d)2;
        equal bit for bit to uploading the dense [S, S, 5] table, tested)."""
        if self.layout != _lib.LAYOUT_STENCIL5:
            raise ValueError("with_stay: STENCIL5 tables only")
        n_tab, A, K, S = self.row_val.shape   # tables held (1 for a shared model), not the instance count
        stay = torch.zeros((n_tab, 1, K, S), dtype=self.row_val.dtype, device=self.row_val.device)
        stay[:, 0, 0, :] = 1.0                                     # slot 0 = the state itself
        row_val = torch.cat([self.row_val, stay], dim=1).contiguous()
        return DeviceMDP(self.layout, S, A + 1, self.batch, self.shared, row_val, width=self.width,
                         height=self.height, device=self.device)

    #: ELL slots per state above which (and above S / 8) a table is kept DENSE
    DENSE_MIN_SLOTS = 32

    @classmethod
    def from_dense(cls, p_transition, device=None, grid=None, layout=None):
        """Upload a dense ``[S, S, A]`` table (one instance, shared layout).

        The STENCIL5 layout is used when every nonzero lies on the stencil of a
        square (or ``grid=(width, height)``) grid; otherwise ELL, or DENSE when
        rows are so full that ELL would gather more than ``DENSE_MIN_SLOTS`` and
        more than S / 8 slots per state.  ``layout`` ("stencil", "ell", "dense")
        forces one (tests; "stencil" still falls back when the table is not a grid).
        """
        device = _lib.require_device(device)
        lib = _lib.load()
        p = np.asarray(p_transition)
        if p.ndim != 3 or p.shape[0] != p.shape[1]:
            raise ValueError(f"p_transition must have shape (S, S, A), got {p.shape}")
        S, _, A = p.shape
        p = np.ascontiguousarray(p, dtype=np.float64)
        if grid is not None:
            w, h = grid
        else:
            w = h = _is_square(S)
        dense = torch.from_numpy(p).to(device)
        if layout == "dense":
            return cls._dense_rows(dense, S, A, device)
        if w and w * h == S and layout != "ell":
            row_val = torch.empty((1, A, 5, S), dtype=torch.float64, device=device)
            flag = torch.zeros(1, dtype=torch.int32, device=device)
            _lib.check(lib.irlmx_dense_to_stencil(_lib.ptr(dense), w, h, A, _lib.ptr(row_val), _lib.ptr(flag),
                                                  _lib.stream_ptr(device)), "dense_to_stencil")
            if not int(flag.item()):
                return cls(_lib.LAYOUT_STENCIL5, S, A, 1, True, row_val, width=w, height=h, device=device)
        return cls._ell_from_dense(dense, S, A, device, allow_dense=layout != "ell")

    @classmethod
    def _dense_rows(cls, dense, S, A, device):
        """DENSE layout of a dense device table (irlmx_dense_to_rows)."""
        lib = _lib.load()
        row_val = torch.empty((1, A, S, S), dtype=torch.float64, device=device)
        col_val = torch.empty((1, S, S), dtype=torch.float64, device=device)
        _lib.check(lib.irlmx_dense_to_rows(_lib.ptr(dense), S, A, _lib.ptr(row_val), _lib.ptr(col_val),
                                           _lib.stream_ptr(device)), "dense_to_rows")
        return cls(_lib.LAYOUT_DENSE, S, A, 1, True, row_val, col_val=col_val, k_row=S, k_col=S, device=device)

    @classmethod
    def resident(cls, p_transition, device=None):
        """:meth:`from_dense` with reuse: the drop-ins (maxent.py, solver.py) call
        this for every dense ``p_transition`` they receive.  The reference copies
        and re-slices the table on every call (maxent.py:98-102, 143, 320;
        solver.py:37); here a float64 ndarray is uploaded and converted once, and
        passing the same array again reuses the device copy after re-reading, on
        the host, every entry the compact table holds (the stencil or ELL pattern:
        S * K * A values, not S^2 * A) -- an in-place edit of any of them uploads
        afresh.  (Entries outside the pattern are zero by construction; making
        one nonzero in place between calls is the one edit not detected: pass a
        new array, or a DeviceMDP.)"""
        p = p_transition
        if not (isinstance(p, np.ndarray) and p.ndim == 3 and p.dtype == np.float64):
            return cls.from_dense(p, device=device)
        device = _lib.require_device(device)
        hit = _RESIDENT.get(id(p))
        if hit is not None and hit.device == device and hit.matches(p):
            return hit.mdp
        mdp = cls.from_dense(p, device=device)
        if mdp.layout == _lib.LAYOUT_DENSE:
            return mdp   # not kept: validating reuse would re-read every entry (the upload's own cost)
        while len(_RESIDENT) >= _RESIDENT_MAX:
            _RESIDENT.pop(next(iter(_RESIDENT)))
        key = id(p)
        _RESIDENT[key] = _Resident(p, mdp, device)
        weakref.finalize(p, _RESIDENT.pop, key, None)
        return mdp

    @classmethod
    def _ell_from_dense(cls, dense, S, A, device, allow_dense=True):
        """ELL row / column forms of a dense device table (irlmx_dense_to_ell), or
        the DENSE layout when the rows are too full for ELL to pay."""
        lib = _lib.load()
        st = _lib.stream_ptr(device)
        k = torch.empty(2, dtype=torch.int32, device=device)
        scratch = torch.empty(S, dtype=torch.int32, device=device)
        _lib.check(lib.irlmx_dense_ell_sizes(_lib.ptr(dense), S, A, _lib.ptr(k), _lib.ptr(scratch), st),
                   "dense_ell_sizes")
        k_row, k_col = (max(1, int(v)) for v in k.tolist())
        if allow_dense and max(k_row, k_col) > cls.DENSE_MIN_SLOTS and 8 * max(k_row, k_col) > S:
            return cls._dense_rows(dense, S, A, device)
        row_idx = torch.empty((1, k_row, S), dtype=torch.int32, device=device)
        row_val = torch.empty((1, A, k_row, S), dtype=torch.float64, device=device)
        col_idx = torch.empty((1, k_col, S), dtype=torch.int32, device=device)
        col_val = torch.empty((1, A, k_col, S), dtype=torch.float64, device=device)
        _lib.check(lib.irlmx_dense_to_ell(_lib.ptr(dense), S, A, k_row, k_col, _lib.ptr(row_idx), _lib.ptr(row_val),
                                          _lib.ptr(col_idx), _lib.ptr(col_val), st), "dense_to_ell")
        return cls(_lib.LAYOUT_ELL, S, A, 1, True, row_val, row_idx=row_idx, col_idx=col_idx, col_val=col_val,
                   k_row=k_row, k_col=k_col, device=device)

    # -- views -------------------------------------------------------------

    def with_batch(self, batch):
        """The same single table applied to ``batch`` instances (shared)."""
        if not self.shared and self.batch != 1:
            raise ValueError("with_batch needs a single-table model")
        return DeviceMDP(self.layout, self.n_states, self.n_actions, batch, True, self.row_val, self.row_idx,
                         self.col_idx, self.col_val, self.width, self.height, self.k_row, self.k_col,
                         self.device)

    def select(self, lo, hi):
        """Instances [lo, hi) of a batched (non-shared) model, as a view."""
        if self.shared:
            return self.with_batch(hi - lo)
        sl = lambda t: t[lo:hi] if t is not None else None
        return DeviceMDP(self.layout, self.n_states, self.n_actions, hi - lo, False, sl(self.row_val),
                         sl(self.row_idx), sl(self.col_idx), sl(self.col_val), self.width, self.height,
                         self.k_row, self.k_col, self.device)

    def take(self, index):
        """Instances ``index`` (int64 device or host indices, in that order) as a
        new model: a shared table is reused as is; per-instance tables are
        gathered into fresh contiguous tensors (irlmx.batch compaction)."""
        index = torch.as_tensor(index, dtype=torch.int64, device=self.device)
        n = int(index.numel())
        if self.shared:
            return self.with_batch(n)
        g = lambda t: t.index_select(0, index).contiguous() if t is not None else None
        return DeviceMDP(self.layout, self.n_states, self.n_actions, n, False, g(self.row_val), g(self.row_idx),
                         g(self.col_idx), g(self.col_val), self.width, self.height, self.k_row, self.k_col,
                         self.device)

    def struct(self):
        """The ``irlmx_mdp`` C struct (pointers stay valid while self is alive)."""
        if self._struct is None:
            s = _lib.MDPStruct()
            s.layout = self.layout
            s.n_states = self.n_states
            s.n_actions = self.n_actions
            s.width = self.width
            s.height = self.height
            s.k_row = self.k_row if self.layout != _lib.LAYOUT_STENCIL5 else 5
            s.k_col = self.k_col if self.layout != _lib.LAYOUT_STENCIL5 else 5
            s.batch = self.batch
            s.shared = 1 if self.shared else 0
            s.row_val = self.row_val.data_ptr()
            s.row_idx = self.row_idx.data_ptr() if self.row_idx is not None else 0
            s.col_idx = self.col_idx.data_ptr() if self.col_idx is not None else 0
            s.col_val = self.col_val.data_ptr() if self.col_val is not None else 0
            # table properties the calls would otherwise re-check on the device
            # per call (irlmx_mdp_properties, one synchronising check per model:
            # the tables of a DeviceMDP are never edited in place): the
            # compact-weight structure at width 256, ELL row order
            lib = _lib.load()
            if hasattr(lib, "irlmx_mdp_properties") and (   # (an older IRLMX_LIB variant build may lack it)
                    self.layout == _lib.LAYOUT_ELL or (self.layout == _lib.LAYOUT_STENCIL5 and self.width == 256)):
                props = ctypes.c_int32(0)
                _lib.check(lib.irlmx_mdp_properties(ctypes.byref(s), ctypes.byref(props),
                                                            _lib.stream_ptr(self.device)), "mdp_properties")
                s.props = props.value
            self._struct = s
        return ctypes.byref(self._struct)

    def pattern(self, b=0):
        """Host index arrays ``(rows, cols)`` [S, K] of every (from, to) pair the
        compact table of instance b stores (off-grid stencil slots clip to the
        state itself)."""
        S = self.n_states
        s = np.arange(S)
        if self.layout == _lib.LAYOUT_STENCIL5:
            x, y = s % self.width, s // self.width
            cols = np.stack([s, np.where(x + 1 < self.width, s + 1, s), np.where(x > 0, s - 1, s),
                             np.where(y + 1 < self.height, s + self.width, s), np.where(y > 0, s - self.width, s)],
                            axis=1)
        else:
            cols = self.row_idx[0 if self.shared else b].cpu().numpy().T.astype(np.int64)
        return np.broadcast_to(s[:, None], cols.shape), cols

    def to_dense(self, b=0):
        """Dense ``[S, S, A]`` numpy table of instance b (tests and small sizes only)."""
        S, A = self.n_states, self.n_actions
        rv = self.row_val[0 if self.shared else b].cpu().numpy()
        if self.layout == _lib.LAYOUT_DENSE:
            return np.ascontiguousarray(np.transpose(rv, (1, 2, 0)))
        out = np.zeros((S, S, A))
        if self.layout == _lib.LAYOUT_STENCIL5:
            s = np.arange(S)
            x, y = s % self.width, s // self.width
            nbrs = [s, np.where(x + 1 < self.width, s + 1, -1), np.where(x > 0, s - 1, -1),
                    np.where(y + 1 < self.height, s + self.width, -1), np.where(y > 0, s - self.width, -1)]
            for k, t in enumerate(nbrs):
                ok = t >= 0
                for a in range(A):
                    out[s[ok], t[ok], a] = rv[a, k, ok]
        else:
            ri = self.row_idx[0 if self.shared else b].cpu().numpy()
            for k in range(self.k_row):
                for a in range(A):
                    np.add.at(out, (np.arange(S), ri[k], a), rv[a, k])
        return out


class _Resident:
    """A dense table's device copy, reused while the caller passes the same,
    unchanged ndarray (weakly referenced: dropped when the array is)."""

    def __init__(self, p, mdp, device):
        self.ref = weakref.ref(p)
        self.device = device
        self.addr = p.__array_interface__["data"][0]
        self.shape, self.strides = p.shape, p.strides
        self.mdp = mdp
        self.rows, self.cols = mdp.pattern()
        self.vals = p[self.rows, self.cols, :].copy()   # every entry the device table holds

    def matches(self, p):
        return (self.ref() is p and p.__array_interface__["data"][0] == self.addr and p.shape == self.shape
                and p.strides == self.strides
                and np.array_equal(p[self.rows, self.cols, :], self.vals, equal_nan=True))


_RESIDENT = {}        # id(ndarray) -> _Resident
_RESIDENT_MAX = 2     # device copies kept (one gridworld table is 1.3 MB at 128x128 in STENCIL5)
