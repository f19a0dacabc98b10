"""osqp_amd -- drop-in for the reference's `osqp.OSQP` on AMD MI355X.

The reference builds sparse MPC QPs in Python and calls OSQP through
``prob = osqp.OSQP(); prob.setup(P, q, A, l, u, **settings)``, ``prob.update(q=, l=, u=)``,
``res = prob.solve()`` and reads ``res.x`` / ``res.info.status``
(vehicle_lateral_mpc_slack_increment.py:118,121,237,248,252,256,269;
Control/MPC/mpc_kinematics.py:194-198; Control/MPC/mpc_dynamics.py:240-244,392-396).
This package mirrors that surface (same names, argument meaning, status strings
and ValueError behaviour) and forwards to the C ABI in include/mpcqp.h
(libmpcqp.so), whose HIP kernels do all numerical work.  There is no CPU
fallback: if the extension or a HIP device is missing, calls raise.

Additions beyond osqp's API (same semantics, batched):
  * ``OSQPBatch`` -- B instances sharing one sparsity pattern, values per instance.
"""
from __future__ import annotations

import ctypes as C
import os
import time
from types import SimpleNamespace

import numpy as np
import scipy.sparse as sparse

__all__ = ["OSQP", "OSQPBatch", "DeviceBatch", "constant", "STATUS", "lib", "LIB_PATH"]

# Diagnostic builds (python-mpc_amd/csrc/Makefile): MPCQP_BUILD=exp adds the kernel variants
# measured and not taken (libmpcqp_exp.so), MPCQP_PHASE_PROF=1 (or MPCQP_BUILD=prof) selects
# the build with in-kernel phase timers (libmpcqp_prof.so), MPCQP_BUILD=skew the barrier-race
# build whose barriers skew the waves (libmpcqp_skew.so, tests/test_skew.py)
_BUILD = os.environ.get("MPCQP_BUILD") or ("prof" if os.environ.get("MPCQP_PHASE_PROF") == "1" else "")
if _BUILD not in ("", "exp", "prof", "skew"):
    raise ImportError(f"MPCQP_BUILD={_BUILD!r}: expected exp, prof or skew")
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                        f"libmpcqp_{_BUILD}.so" if _BUILD else "libmpcqp.so")
OSQP_INFTY = 1e30

STATUS = {
    4: "dual infeasible inaccurate",
    3: "primal infeasible inaccurate",
    2: "solved inaccurate",
    1: "solved",
    -2: "maximum iterations reached",
    -3: "primal infeasible",
    -4: "dual infeasible",
    -5: "interrupted",
    -6: "run time limit reached",
    -7: "problem non convex",
    -10: "unsolved",
}

_CONSTANTS = {
    "OSQP_INFTY": OSQP_INFTY, "OSQP_NAN": float("nan"),
    "OSQP_SOLVED": 1, "OSQP_SOLVED_INACCURATE": 2, "OSQP_MAX_ITER_REACHED": -2,
    "OSQP_PRIMAL_INFEASIBLE": -3, "OSQP_PRIMAL_INFEASIBLE_INACCURATE": 3,
    "OSQP_DUAL_INFEASIBLE": -4, "OSQP_DUAL_INFEASIBLE_INACCURATE": 4,
    "OSQP_NON_CVX": -7, "OSQP_UNSOLVED": -10,
}


def constant(name):
    """osqp.constant(name)"""
    if name not in _CONSTANTS:
        raise ValueError("Constant not recognized")
    return _CONSTANTS[name]


class _Settings(C.Structure):
    _fields_ = [
        ("rho", C.c_double), ("sigma", C.c_double), ("alpha", C.c_double),
        ("eps_abs", C.c_double), ("eps_rel", C.c_double),
        ("eps_prim_inf", C.c_double), ("eps_dual_inf", C.c_double),
        ("adaptive_rho_tolerance", C.c_double),
        ("max_iter", C.c_int32), ("scaling", C.c_int32), ("check_termination", C.c_int32),
        ("warm_start", C.c_int32), ("adaptive_rho", C.c_int32),
        ("adaptive_rho_interval", C.c_int32), ("scaled_termination", C.c_int32),
        ("polish", C.c_int32), ("verbose", C.c_int32),
        ("delta", C.c_double), ("polish_refine_iter", C.c_int32),
    ]


class _PlanInfo(C.Structure):
    _fields_ = [
        ("n", C.c_int32), ("m", C.c_int32), ("nb", C.c_int32), ("block", C.c_int32),
        ("npad", C.c_int32), ("max_level", C.c_int32), ("batch", C.c_int64),
        ("n_devices", C.c_int32), ("lds_bytes_solve", C.c_int64), ("bytes_per_instance", C.c_int64),
        ("amax", C.c_int32), ("gather_k", C.c_int32), ("variant", C.c_int32), ("threads_per_qp", C.c_int32),
        ("n_eliminated", C.c_int32), ("plan_choice", C.c_int32),
    ]


_lib = None
_P = C.POINTER


def lib():
    """Load libmpcqp.so (fails loudly if the HIP extension was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} not found: build the HIP extension first "
            "(python -c 'import __graft_entry__ as g; g.build()')")
    # One HIP runtime per process: torch wheels ship their own libamdhip64 (same soname
    # as /opt/rocm's).  Loaded first, torch's copy also satisfies libmpcqp.so's
    # dependency; loaded the other way round the process ends up with two runtimes and
    # torch.cuda sees no device.  Device tensors are handed to the C ABI (DeviceBatch,
    # mpc_device), so torch goes first whenever it is installed.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    i32p, dp, vp = _P(C.c_int32), _P(C.c_double), C.c_void_p
    hp = _P(C.c_void_p)
    L.mpcqp_default_settings.argtypes = [_P(_Settings)]
    L.mpcqp_default_settings.restype = None
    L.mpcqp_last_error.restype = C.c_char_p
    L.mpcqp_setup_batch.argtypes = [C.c_int32, C.c_int32, i32p, i32p, i32p, i32p, C.c_int64,
                                    dp, dp, dp, dp, dp, _P(_Settings), C.c_uint32, hp]
    L.mpcqp_update_batch.argtypes = [vp, dp, dp, dp]
    L.mpcqp_update_settings.argtypes = [vp, _P(_Settings), C.c_int32]
    L.mpcqp_update_matrices_batch.argtypes = [vp, dp, i32p, C.c_int32, dp, i32p, C.c_int32]
    L.mpcqp_warm_start_batch.argtypes = [vp, dp, dp]
    L.mpcqp_solve_batch.argtypes = [vp, dp, dp, i32p, i32p]
    L.mpcqp_get_info_batch.argtypes = [vp, dp, dp, dp, dp, i32p]
    L.mpcqp_get_certificates.argtypes = [vp, dp, dp]
    L.mpcqp_get_polish_status.argtypes = [vp, i32p]
    L.mpcqp_create.argtypes = [C.c_int32, C.c_int32, i32p, i32p, i32p, i32p, C.c_int64,
                               _P(_Settings), C.c_int32, hp]
    L.mpcqp_setup_device.argtypes = [vp, vp, vp, vp, vp, vp, vp]
    L.mpcqp_update_device.argtypes = [vp, vp, vp, vp, vp]
    L.mpcqp_setup_solve_device.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.mpcqp_warm_start_device.argtypes = [vp, vp, vp, vp]
    L.mpcqp_setup_warm_device.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.mpcqp_setup_warm_fused.argtypes = [vp]
    L.mpcqp_solve_device.argtypes = [vp, vp, vp, vp, vp, vp]
    L.mpcqp_synchronize.argtypes = [vp]
    L.mpcqp_set_shared_matrices.argtypes = [vp, C.c_int32]
    L.mpcqp_set_one_shot.argtypes = [vp, C.c_int32]
    L.mpcqp_one_shot_applies.argtypes = [vp]
    L.mpcqp_get_stream.argtypes = [vp]
    L.mpcqp_get_stream.restype = vp
    L.mpcqp_last_kernel_ms.argtypes = [vp]
    L.mpcqp_last_kernel_ms.restype = C.c_double
    L.mpcqp_get_plan_info.argtypes = [vp, _P(_PlanInfo)]
    L.mpcqp_timing.argtypes = [vp, C.c_int32]
    L.mpcqp_timing_read.argtypes = [vp, dp, i32p, dp, i32p]
    L.mpcqp_debug_phase_times.argtypes = [vp, _P(C.c_int64)]
    L.mpcqp_debug_dispatch_order.argtypes = [vp, _P(C.c_int32)]
    L.mpcqp_debug_copy.argtypes = [vp, vp, C.c_int64, C.c_int32, vp, dp]
    L.mpcqp_free.argtypes = [vp]
    L.mpcqp_free.restype = None
    L.mpcqp_analyze.argtypes = [C.c_int32, C.c_int32, i32p, i32p, i32p, i32p,
                                i32p, i32p, i32p, i32p]
    L.mpcqp_analyze_ex.argtypes = [C.c_int32, C.c_int32, i32p, i32p, i32p, i32p, C.c_int32,
                                   i32p, i32p, i32p, i32p, i32p]
    L.mpcqp_plan_preview.argtypes = [C.c_int32, C.c_int32, i32p, i32p, i32p, i32p, _P(_Settings),
                                     _P(_PlanInfo), C.c_char_p, C.c_int32]
    _lib = L
    return L


def _dp(a):
    return None if a is None else a.ctypes.data_as(_P(C.c_double))


def _ip(a):
    return None if a is None else a.ctypes.data_as(_P(C.c_int32))


def _check(code, what):
    if code:
        msg = lib().mpcqp_last_error().decode()
        if code in (1, 5):  # invalid data; non-convex P (osqp-python raises ValueError at setup)
            raise ValueError(f"{what}: {msg}")
        if code == 2:
            raise NotImplementedError(f"{what}: {msg}")
        raise RuntimeError(f"{what}: {msg} (code {code})")


_SETTING_NAMES = {f[0] for f in _Settings._fields_}
_IGNORED = {"linsys_solver", "time_limit", "adaptive_rho_fraction"}
# osqp-python 0.6 update_settings: what may change after setup (verbose / time_limit: accepted, no effect)
_UPDATABLE = {"max_iter", "eps_abs", "eps_rel", "eps_prim_inf", "eps_dual_inf", "rho", "alpha", "delta", "polish",
              "polish_refine_iter", "verbose", "scaled_termination", "check_termination", "warm_start", "time_limit"}


def _make_settings(**kw) -> _Settings:
    s = _Settings()
    lib().mpcqp_default_settings(C.byref(s))
    for k, v in kw.items():
        if k in _IGNORED:
            continue
        if k not in _SETTING_NAMES:
            raise ValueError(f"Unrecognized setting {k}")
        if isinstance(v, bool):
            v = int(v)
        setattr(s, k, type(getattr(s, k))(v))
    return s


def _csc_sorted(M):
    """M as CSC with sorted int32-range indices (a copy where scipy would make one)."""
    M = M if sparse.isspmatrix_csc(M) else sparse.csc_matrix(M)
    if not M.has_sorted_indices:
        M = M.copy()
        M.sort_indices()
    return M


def canonical_data(P, A):
    """osqp-python's prepare_data: P -> triu CSC, A -> CSC, sorted int32 indices.  The upper
    triangle is taken from the CSC arrays directly: the same entries and order as
    scipy.sparse.triu (a few tens of microseconds instead of a few hundred on the reference's
    fresh-object-per-call pattern, Control/MPC/mpc_dynamics.py:392).  Duplicate entries of P
    are summed first, as triu's COO -> CSC conversion sums them; A keeps its duplicates, as
    osqp-python passes A's stored entries to OSQP unchanged."""
    if P is None:
        raise ValueError("P must be provided")
    P = _csc_sorted(P)
    if not P.has_canonical_format:  # duplicates (sorted indices are known by now)
        P = P.copy()
        P.sum_duplicates()
    A = _csc_sorted(A)
    n = P.shape[1]
    cols = np.repeat(np.arange(n, dtype=np.int64), np.diff(P.indptr))
    keep = P.indices <= cols
    if not keep.all():
        ptr = np.zeros(n + 1, dtype=P.indptr.dtype)
        np.cumsum(np.bincount(cols[keep], minlength=n), out=ptr[1:])
        P = sparse.csc_matrix((P.data[keep], P.indices[keep], ptr), shape=P.shape)
        P.has_sorted_indices = True
    return P, A


def analyze(P, A, eliminate=False):
    """Host-only symbolic analysis (no GPU): returns (nb, block, var_pad, bsize), and with
    `eliminate` (the plan of the four-wave kernel: degree <= 1 vertices of K taken out of
    the blocks, padded indices from nb * block on) also the number eliminated."""
    P, A = canonical_data(P, A)
    n, m = P.shape[0], A.shape[0]
    nb = C.c_int32(); blk = C.c_int32(); ne = C.c_int32()
    vp = np.empty(n, np.int32); bs = np.empty(max(n, 1), np.int32)
    Pp = np.ascontiguousarray(P.indptr, np.int32); Pi = np.ascontiguousarray(P.indices, np.int32)
    Ap = np.ascontiguousarray(A.indptr, np.int32); Ai = np.ascontiguousarray(A.indices, np.int32)
    _check(lib().mpcqp_analyze_ex(n, m, _ip(Pp), _ip(Pi), _ip(Ap), _ip(Ai), int(eliminate), C.byref(nb),
                                  C.byref(blk), _ip(vp), _ip(bs), C.byref(ne)), "analyze")
    out = (nb.value, blk.value, vp, bs[: nb.value].copy())
    return out + (ne.value,) if eliminate else out


def plan_preview(P, A, **settings):
    """Host-only (no GPU): the plan and solve-kernel variant a batch with this pattern and
    these settings would take (mpcqp_plan_preview) -- plan_info's shape fields, plus
    "note": why an eliminated plan was rejected ("" when it was not)."""
    P, A = canonical_data(P, A)
    n, m = P.shape[0], A.shape[0]
    Pp = np.ascontiguousarray(P.indptr, np.int32); Pi = np.ascontiguousarray(P.indices, np.int32)
    Ap = np.ascontiguousarray(A.indptr, np.int32); Ai = np.ascontiguousarray(A.indices, np.int32)
    s = _make_settings(**{k: v for k, v in settings.items() if k != "verbose"})
    info = _PlanInfo()
    note = C.create_string_buffer(512)
    _check(lib().mpcqp_plan_preview(n, m, _ip(Pp), _ip(Pi), _ip(Ap), _ip(Ai), C.byref(s), C.byref(info),
                                    note, 512), "plan_preview")
    out = {f[0]: getattr(info, f[0]) for f in _PlanInfo._fields_}
    out["note"] = note.value.decode()
    return out


def _keep_mask(V):
    """The value indices of the user's pattern that are nonzero in some instance."""
    V = np.asarray(V)
    return (V != 0).any(axis=0) if V.shape[0] > 1 else V[0] != 0


def _kept_index(V, keep=None):
    """Per value index of the user's pattern: its index once the entries zero in every
    instance are dropped (_drop_common_zeros), or -1."""
    keep = _keep_mask(V) if keep is None else keep
    out = np.full(keep.size, -1, np.int64)
    out[keep] = np.arange(int(keep.sum()))
    return out


def _drop_common_zeros(M, V, keep=None):
    """Entries zero in every instance dropped from the pattern M (CSC, sorted) and from the
    values V (B x nnz), without scipy's copies (the kept entries keep their order)."""
    V = np.asarray(V)
    keep = _keep_mask(V) if keep is None else keep
    if keep.all():
        return M, V
    n = M.shape[1]
    cols = np.repeat(np.arange(n, dtype=np.int64), np.diff(M.indptr))
    ptr = np.zeros(n + 1, dtype=M.indptr.dtype)
    np.cumsum(np.bincount(cols[keep], minlength=n), out=ptr[1:])
    M2 = sparse.csc_matrix((np.ones(int(keep.sum())), M.indices[keep], ptr), shape=M.shape)
    M2.has_sorted_indices = True
    return M2, V[:, keep]


class _Handle:
    def __init__(self, ptr):
        self.ptr = ptr

    def __del__(self):
        if self.ptr:
            lib().mpcqp_free(self.ptr)
            self.ptr = None


class OSQPBatch:
    """B QPs with one shared sparsity pattern, solved together on the GPU(s).

    setup(P, q, A, l, u, Px=None, Ax=None, device_mask=1, **settings):
      P, A  -- scipy sparse templates (pattern; values used when Px/Ax are None)
      q     -- (B, n);  l, u -- (B, m)
      Px    -- (B, nnz(triu(P))) per-instance values in triu(P).tocsc() order
      Ax    -- (B, nnz(A))       per-instance values in A.tocsc() order
    """

    def __init__(self):
        self._h = None
        self.n = self.m = self.B = 0

    def setup(self, P, q, A, l, u, Px=None, Ax=None, device_mask=1, **settings):
        t0 = time.perf_counter()
        P, A = canonical_data(P, A)
        n, m = P.shape[0], A.shape[0]
        if P.shape != (n, n) or A.shape[1] != n:
            raise ValueError("Matrix dimensions are not consistent")
        q = np.atleast_2d(np.asarray(q, np.float64))
        B = q.shape[0]
        l = np.atleast_2d(np.asarray(l, np.float64))
        u = np.atleast_2d(np.asarray(u, np.float64))
        if q.shape != (B, n) or l.shape != (B, m) or u.shape != (B, m):
            raise ValueError("q, l, u must have shapes (B, n), (B, m), (B, m)")
        Px = np.broadcast_to(P.data if Px is None else np.asarray(Px, np.float64), (B, P.nnz))
        Ax = np.broadcast_to(A.data if Ax is None else np.asarray(Ax, np.float64), (B, A.nnz))
        # Entries that are zero in every instance contribute exactly 0 to every OSQP
        # operation, so dropping them is bit-for-bit neutral; it keeps structural
        # zeros of the reference's assembly (e.g. C~'QC~ at mpc_dynamics.py:296-297)
        # out of the sparsity plan.
        # user value index -> index in the kept pattern (-1: dropped), for update(Px_idx=, Ax_idx=)
        # (the index maps are formed on the first update(Px=/Ax=), not at every setup)
        kp, ka = _keep_mask(Px), _keep_mask(Ax)
        self._keep = (kp, ka)
        self._pmap = self._amap = None
        self._nnz_user = (P.nnz, A.nnz)
        P, Px = _drop_common_zeros(P, Px, kp)
        A, Ax = _drop_common_zeros(A, Ax, ka)
        Px = np.ascontiguousarray(Px, np.float64)
        Ax = np.ascontiguousarray(Ax, np.float64)
        q = np.ascontiguousarray(q); l = np.ascontiguousarray(l); u = np.ascontiguousarray(u)
        self._pattern = (np.ascontiguousarray(P.indptr, np.int32), np.ascontiguousarray(P.indices, np.int32),
                         np.ascontiguousarray(A.indptr, np.int32), np.ascontiguousarray(A.indices, np.int32))
        Pp, Pi, Ap, Ai = self._pattern
        s = _make_settings(**settings)
        self._settings = s
        self._settings_kw = dict(settings)
        h = C.c_void_p()
        _check(lib().mpcqp_setup_batch(n, m, _ip(Pp), _ip(Pi), _ip(Ap), _ip(Ai), B, _dp(Px), _dp(Ax),
                                       _dp(q), _dp(l), _dp(u), C.byref(s), int(device_mask), C.byref(h)),
               "setup")
        self._h = _Handle(h.value)
        self.n, self.m, self.B = n, m, B
        self.setup_time = time.perf_counter() - t0

    def _need(self):
        if self._h is None:
            raise ValueError("Workspace not initialized!")
        return self._h.ptr

    def update(self, q=None, l=None, u=None, Px=None, Px_idx=None, Ax=None, Ax_idx=None):
        """osqp-python 0.6's update order: q, the bounds, then the matrices.  Px: (B, k)
        values of triu(P) at Px_idx (k indices into the setup's triu(P).tocsc() value array;
        None or empty: all nnz), likewise Ax / Ax_idx (mpcqp_update_matrices_batch)."""
        h = self._need()
        if q is None and l is None and u is None and Px is None and Ax is None:
            raise ValueError("No updatable data has been specified!")
        B, n, m = self.B, self.n, self.m
        if q is not None or l is not None or u is not None:
            self._update_vectors(h, q, l, u)
        if Px is not None or Ax is not None:
            if self._pmap is None:
                self._pmap, self._amap = _kept_index(None, self._keep[0]), _kept_index(None, self._keep[1])
            P = self._matrix_values(Px, Px_idx, self._pmap, self._nnz_user[0], "P")
            A = self._matrix_values(Ax, Ax_idx, self._amap, self._nnz_user[1], "A")
            pv, pi = P if P else (None, None)
            av, ai = A if A else (None, None)
            _check(lib().mpcqp_update_matrices_batch(
                h, _dp(pv), None if pi is None else _ip(pi), 0 if pi is None else len(pi),
                _dp(av), None if ai is None else _ip(ai), 0 if ai is None else len(ai)), "update matrices")

    def _matrix_values(self, V, idx, kmap, nnz_user, name):
        """(values (B, k') in the kept pattern, kept indices (k',)) for the library, or None.
        A value for an entry that was zero in every instance at setup (dropped from the
        pattern) must stay zero: the pattern is fixed."""
        if V is None:
            return None
        B = self.B
        V = np.asarray(V, np.float64)
        if idx is None or np.size(idx) == 0:
            V = V.reshape(B, nnz_user)
            idx = np.arange(nnz_user)
        else:
            idx = np.asarray(idx).ravel().astype(np.int64)
            if idx.size > nnz_user:
                raise ValueError(f"new number of elements ({idx.size}) greater than elements in {name} ({nnz_user})")
            if idx.min() < 0 or idx.max() >= nnz_user:
                raise ValueError(f"{name}x_idx out of range")
            V = V.reshape(B, idx.size)
        kept = kmap[idx]
        dropped = kept < 0
        if np.any(V[:, dropped] != 0):
            raise ValueError(f"{name}x sets an entry that was zero in every instance at setup "
                             "(not in the sparsity pattern); run setup() again")
        return (np.ascontiguousarray(V[:, ~dropped]), np.ascontiguousarray(kept[~dropped], np.int32))

    def _update_vectors(self, h, q, l, u):
        B, n, m = self.B, self.n, self.m

        def prep(v, k, clip):
            if v is None:
                return None
            v = np.asarray(v, np.float64).reshape(B, k)
            if clip is not None:
                v = np.maximum(v, -OSQP_INFTY) if clip < 0 else np.minimum(v, OSQP_INFTY)
            return np.ascontiguousarray(v)

        q = prep(q, n, None); l = prep(l, m, -1); u = prep(u, m, 1)
        _check(lib().mpcqp_update_batch(h, _dp(q), _dp(l), _dp(u)), "update")

    def update_settings(self, **kw):
        """osqp.OSQP.update_settings (mpcqp_update_settings): max_iter, eps_*, rho, alpha, delta,
        polish, polish_refine_iter, scaled_termination, check_termination, warm_start."""
        h = self._need()
        bad = sorted(set(kw) - _UPDATABLE)
        if bad:
            raise ValueError(f"setting(s) {', '.join(bad)} cannot be changed after setup")
        new = dict(self._settings_kw, **kw)
        s = _make_settings(**new)
        _check(lib().mpcqp_update_settings(h, C.byref(s), int("rho" in kw)), "update_settings")
        self._settings, self._settings_kw = s, new

    def warm_start(self, x=None, y=None):
        h = self._need()
        x = None if x is None else np.ascontiguousarray(np.asarray(x, np.float64).reshape(self.B, self.n))
        y = None if y is None else np.ascontiguousarray(np.asarray(y, np.float64).reshape(self.B, self.m))
        _check(lib().mpcqp_warm_start_batch(h, _dp(x), _dp(y)), "warm_start")
        self._settings_kw["warm_start"] = True  # (osqp_warm_start turns the setting on)

    def solve(self):
        h = self._need()
        B, n, m = self.B, self.n, self.m
        x = np.empty((B, n)); y = np.empty((B, m))
        st = np.empty(B, np.int32); it = np.empty(B, np.int32)
        t0 = time.perf_counter()
        _check(lib().mpcqp_solve_batch(h, _dp(x), _dp(y), _ip(st), _ip(it)), "solve")
        solve_time = time.perf_counter() - t0
        obj = np.empty(B); pri = np.empty(B); dua = np.empty(B); rho = np.empty(B)
        ru = np.empty(B, np.int32)
        _check(lib().mpcqp_get_info_batch(h, _dp(obj), _dp(pri), _dp(dua), _dp(rho), _ip(ru)), "info")
        pc = np.empty((B, m)); dc = np.empty((B, n))
        _check(lib().mpcqp_get_certificates(h, _dp(pc), _dp(dc)), "certificates")
        sp = np.empty(B, np.int32)
        _check(lib().mpcqp_get_polish_status(h, _ip(sp)), "polish status")
        return SimpleNamespace(x=x, y=y, status_val=st, iter=it, obj_val=obj, pri_res=pri, dua_res=dua,
                               rho_estimate=rho, rho_updates=ru, prim_inf_cert=pc, dual_inf_cert=dc,
                               status_polish=sp, solve_time=solve_time,
                               status=[STATUS.get(int(v), "unknown") for v in st])

    def plan_info(self):
        info = _PlanInfo()
        _check(lib().mpcqp_get_plan_info(self._need(), C.byref(info)), "plan_info")
        return {f[0]: getattr(info, f[0]) for f in _PlanInfo._fields_}

    def phase_times(self):
        """Per-instance phase timers of the last solve, shape (B, 24) int64 (diagnostic;
        needs MPCQP_PHASE_PROF=1 in the environment before setup)."""
        out = np.zeros((self.B, 24), dtype=np.int64)
        _check(lib().mpcqp_debug_phase_times(self._need(), out.ctypes.data_as(_P(C.c_int64))), "phase_times")
        return out


class OSQP:
    """Single-instance mirror of osqp.OSQP (runs as a batch of one on the GPU)."""

    def __init__(self):
        self._b = None

    def setup(self, P=None, q=None, A=None, l=None, u=None, **settings):
        if P is None or A is None:
            raise ValueError("P and A must be provided")
        n = P.shape[0]
        m = A.shape[0]
        q = np.zeros(n) if q is None else np.asarray(q, np.float64).ravel()
        l = np.full(m, -np.inf) if l is None else np.asarray(l, np.float64).ravel()
        u = np.full(m, np.inf) if u is None else np.asarray(u, np.float64).ravel()
        if len(q) != n:
            raise ValueError("Incorrect dimension of q")
        if len(l) != m or len(u) != m:
            raise ValueError("Incorrect dimension of l or u")
        l = np.maximum(l, -OSQP_INFTY)
        u = np.minimum(u, OSQP_INFTY)
        self._settings_kw = dict(settings)
        self._b = OSQPBatch()
        self._b.setup(P, q[None, :], A, l[None, :], u[None, :], **settings)
        self._update_time = 0.0

    def update(self, q=None, l=None, u=None, Px=None, Px_idx=np.array([]), Ax=None, Ax_idx=np.array([])):
        if self._b is None:
            raise ValueError("Workspace not initialized!")
        n, m = self._b.n, self._b.m
        if q is not None and len(q) != n:
            raise ValueError("q must have length n")
        if l is not None:
            if not isinstance(l, np.ndarray):
                raise TypeError("l must be numpy.ndarray, not %s" % type(l).__name__)
            if len(l) != m:
                raise ValueError("l must have length m")
        if u is not None:
            if not isinstance(u, np.ndarray):
                raise TypeError("u must be numpy.ndarray, not %s" % type(u).__name__)
            if len(u) != m:
                raise ValueError("u must have length m")
        t0 = time.perf_counter()
        self._b.update(q=None if q is None else np.asarray(q, np.float64)[None, :],
                       l=None if l is None else l[None, :], u=None if u is None else u[None, :],
                       Px=None if Px is None else np.asarray(Px, np.float64)[None, :], Px_idx=Px_idx,
                       Ax=None if Ax is None else np.asarray(Ax, np.float64)[None, :], Ax_idx=Ax_idx)
        self._update_time = time.perf_counter() - t0

    def update_settings(self, **kwargs):
        if self._b is None:
            raise ValueError("Workspace not initialized!")
        self._b.update_settings(**kwargs)

    def warm_start(self, x=None, y=None):
        if self._b is None:
            raise ValueError("Workspace not initialized!")
        self._b.warm_start(x=x, y=y)

    def solve(self):
        if self._b is None:
            raise ValueError("Workspace not initialized!")
        r = self._b.solve()
        sv = int(r.status_val[0])
        info = SimpleNamespace(
            iter=int(r.iter[0]), status=STATUS.get(sv, "unknown"), status_val=sv,
            status_polish=int(r.status_polish[0]),
            obj_val=float(r.obj_val[0]), pri_res=float(r.pri_res[0]), dua_res=float(r.dua_res[0]),
            setup_time=self._b.setup_time, solve_time=r.solve_time, update_time=self._update_time,
            polish_time=0.0, run_time=r.solve_time, rho_updates=int(r.rho_updates[0]),
            rho_estimate=float(r.rho_estimate[0]))
        return SimpleNamespace(x=r.x[0], y=r.y[0], info=info, prim_inf_cert=r.prim_inf_cert[0],
                               dual_inf_cert=r.dual_inf_cert[0], dua_inf_cert=r.dual_inf_cert[0])


class DeviceBatch:
    """Device-resident batch on one GPU: inputs and outputs stay in HBM.

    Thin wrapper over mpcqp_create / mpcqp_setup_device / mpcqp_solve_device for
    callers that keep their data on the device (bench.py; a future on-device
    QP assembly).  Arrays are any objects exposing
    ``data_ptr()`` to contiguous float64 / int32 device memory on `device`
    (e.g. torch tensors); this module never touches their contents.
    P, A give the shared pattern (canonicalised like osqp-python; values ignored).
    ``stream``: a hipStream_t (int or c_void_p); None = the handle's own stream, which
    is NOT ordered with torch's legacy default stream -- callers mixing torch kernels
    and these calls pass a non-default torch stream's ``cuda_stream`` (see
    mpc_device.DynamicMPC) or synchronise in between.
    """

    def __init__(self, P, A, B, device=0, **settings):
        P, A = canonical_data(P, A)
        self.n, self.m, self.B = P.shape[0], A.shape[0], int(B)
        self.nnzP, self.nnzA = P.nnz, A.nnz
        self._pattern = (np.ascontiguousarray(P.indptr, np.int32), np.ascontiguousarray(P.indices, np.int32),
                         np.ascontiguousarray(A.indptr, np.int32), np.ascontiguousarray(A.indices, np.int32))
        Pp, Pi, Ap, Ai = self._pattern
        s = _make_settings(**settings)
        h = C.c_void_p()
        _check(lib().mpcqp_create(self.n, self.m, _ip(Pp), _ip(Pi), _ip(Ap), _ip(Ai), self.B, C.byref(s),
                                  int(device), C.byref(h)), "create")
        self._h = _Handle(h.value)

    @staticmethod
    def _ptr(t):
        return None if t is None else C.c_void_p(t.data_ptr())

    def _shared(self, Px, Ax):
        """1-D Px / Ax: one P and A for every instance (LTI batches; mpcqp_set_shared_matrices)."""
        shared = Px.dim() == 1
        if shared != (Ax.dim() == 1):
            raise ValueError("Px and Ax must both be per-instance (2-D) or both shared (1-D)")
        if shared and (Px.shape[0] != self.nnzP or Ax.shape[0] != self.nnzA):
            raise ValueError("shared Px / Ax must have nnz(P) / nnz(A) entries")
        _check(lib().mpcqp_set_shared_matrices(self._h.ptr, int(shared)), "set_shared_matrices")

    def setup(self, Px, Ax, q, l, u, stream=None):
        self._shared(Px, Ax)
        _check(lib().mpcqp_setup_device(self._h.ptr, self._ptr(Px), self._ptr(Ax), self._ptr(q), self._ptr(l),
                                        self._ptr(u), stream), "setup_device")

    def update(self, q=None, l=None, u=None, stream=None):
        _check(lib().mpcqp_update_device(self._h.ptr, self._ptr(q), self._ptr(l), self._ptr(u), stream),
               "update_device")

    def warm_start(self, x=None, y=None, stream=None):
        _check(lib().mpcqp_warm_start_device(self._h.ptr, self._ptr(x), self._ptr(y), stream), "warm_start_device")

    def setup_warm(self, Px, Ax, q, l, u, x=None, y=None, stream=None):
        """setup(Px, Ax, q, l, u) then warm_start(x, y) -- one fused kernel where the wide batch
        setup applies (mpcqp_setup_warm_device; setup_warm_fused()), identical results."""
        self._shared(Px, Ax)
        _check(lib().mpcqp_setup_warm_device(self._h.ptr, self._ptr(Px), self._ptr(Ax), self._ptr(q), self._ptr(l),
                                             self._ptr(u), self._ptr(x), self._ptr(y), stream), "setup_warm_device")

    def setup_warm_fused(self):
        """1 when setup_warm runs as one kernel for this handle's plan (mpcqp_setup_warm_fused)."""
        return int(lib().mpcqp_setup_warm_fused(self._h.ptr))

    def solve(self, x=None, y=None, status=None, iters=None, stream=None):
        _check(lib().mpcqp_solve_device(self._h.ptr, self._ptr(x), self._ptr(y), self._ptr(status),
                                        self._ptr(iters), stream), "solve_device")

    def setup_solve(self, Px, Ax, q, l, u, x=None, y=None, status=None, iters=None, stream=None):
        """setup(Px, Ax, q, l, u) then solve(x, y, status, iters) -- one fused kernel where the
        solve kernel allows it (mpcqp_setup_solve_device), identical results.  Px / Ax 1-D:
        one P and A shared by the batch (LTI layouts)."""
        self._shared(Px, Ax)
        _check(lib().mpcqp_setup_solve_device(self._h.ptr, self._ptr(Px), self._ptr(Ax), self._ptr(q), self._ptr(l),
                                              self._ptr(u), self._ptr(x), self._ptr(y), self._ptr(status),
                                              self._ptr(iters), stream), "setup_solve_device")

    def one_shot(self, on=True):
        """mpcqp_set_one_shot: setup_solve keeps no workspace state (the scaled problem, the G
        blocks, the warm-start iterates, the certificates) for later calls -- the Control/MPC
        pattern of a fresh setup() + solve() per call.  Returns the form that applies to this
        handle's kernel: 0 none (not the fused four-wave kernel), 1 the G blocks in the workspace,
        2 in an LDS region of their own, 3 straight into the solve's LDS copy
        (mpcqp_one_shot_applies)."""
        _check(lib().mpcqp_set_one_shot(self._h.ptr, int(on)), "set_one_shot")
        return int(lib().mpcqp_one_shot_applies(self._h.ptr))

    def synchronize(self):
        _check(lib().mpcqp_synchronize(self._h.ptr), "synchronize")

    def stream_handle(self):
        """The handle's own HIP stream (what stream=None means), for work the caller wants
        ordered with the handle's calls without a synchronisation."""
        return C.c_void_p(lib().mpcqp_get_stream(self._h.ptr))

    def timing(self, enable=True, setup=True):
        """HIP-event timing of the solve launches (and of the setup launches when
        `setup`); every recorded event is one more packet between the kernels."""
        mask = (1 | (2 if setup else 0)) if enable else 0
        _check(lib().mpcqp_timing(self._h.ptr, mask), "timing")

    def timing_read(self):
        sm = C.c_double(); so = C.c_double(); ns = C.c_int32(); no = C.c_int32()
        _check(lib().mpcqp_timing_read(self._h.ptr, C.byref(sm), C.byref(ns), C.byref(so), C.byref(no)), "timing")
        return dict(setup_ms=sm.value, n_setup=ns.value, solve_ms=so.value, n_solve=no.value)

    def plan_info(self):
        info = _PlanInfo()
        _check(lib().mpcqp_get_plan_info(self._h.ptr, C.byref(info)), "plan_info")
        return {f[0]: getattr(info, f[0]) for f in _PlanInfo._fields_}

    def phase_times(self):
        """Per-instance phase timers of the last solve, shape (B, 24) int64 (diagnostic;
        needs MPCQP_PHASE_PROF=1 in the environment when the batch was created)."""
        out = np.zeros((self.B, 24), dtype=np.int64)
        _check(lib().mpcqp_debug_phase_times(self._h.ptr, out.ctypes.data_as(_P(C.c_int64))), "phase_times")
        return out

    def dispatch_order(self):
        """The dispatch order the next solve uses, shape (B,) int32 (diagnostic; see
        mpcqp.h::mpcqp_debug_dispatch_order)."""
        out = np.zeros(self.B, dtype=np.int32)
        _check(lib().mpcqp_debug_dispatch_order(self._h.ptr, out.ctypes.data_as(_P(C.c_int32))), "dispatch_order")
        return out
