"""ctypes binding of the CPU oracle (oracle/liboracle.so) -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  It mirrors the `osqp.OSQP` Python surface the reference uses
(vehicle_lateral_mpc_slack_increment.py:118,121,237,248,269;
Control/MPC/mpc_dynamics.py:392-396) so parity tests read like the reference's
own call pattern.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from types import SimpleNamespace

import numpy as np
import scipy.sparse as sparse

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")

STATUS_STR = {
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


class _Settings(C.Structure):
    _fields_ = [
        ("rho", C.c_double), ("sigma", C.c_double), ("alpha", C.c_double),
        ("eps_abs", C.c_double), ("eps_rel", C.c_double),
        ("eps_prim_inf", C.c_double), ("eps_dual_inf", C.c_double),
        ("adaptive_rho_tolerance", C.c_double), ("adaptive_rho_fraction", C.c_double),
        ("max_iter", C.c_int), ("scaling", C.c_int), ("check_termination", C.c_int),
        ("warm_start", C.c_int), ("adaptive_rho", C.c_int),
        ("adaptive_rho_interval", C.c_int), ("scaled_termination", C.c_int),
        ("delta", C.c_double), ("polish", C.c_int), ("polish_refine_iter", C.c_int),
    ]


class _Info(C.Structure):
    _fields_ = [
        ("iter", C.c_int), ("status_val", C.c_int), ("rho_updates", C.c_int),
        ("obj_val", C.c_double), ("pri_res", C.c_double), ("dua_res", C.c_double),
        ("rho_estimate", C.c_double), ("status_polish", C.c_int),
    ]


def build(force: bool = False) -> str:
    src = os.path.join(_HERE, "osqp_oracle.c")
    if force or not os.path.exists(_LIB) or os.path.getmtime(_LIB) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE, "liboracle.so"])
    return _LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = C.CDLL(_LIB)
        P = C.POINTER
        L.orc_default_settings.argtypes = [P(_Settings)]
        L.orc_setup.argtypes = [P(C.c_void_p), C.c_int, C.c_int,
                                P(C.c_int), P(C.c_int), P(C.c_double), P(C.c_double),
                                P(C.c_int), P(C.c_int), P(C.c_double),
                                P(C.c_double), P(C.c_double), P(_Settings)]
        for name in ("orc_update_lin_cost", "orc_update_lower_bound", "orc_update_upper_bound"):
            getattr(L, name).argtypes = [C.c_void_p, P(C.c_double)]
        L.orc_update_bounds.argtypes = [C.c_void_p, P(C.c_double), P(C.c_double)]
        L.orc_update_settings.argtypes = [C.c_void_p, P(_Settings), C.c_int]
        L.orc_update_P_A.argtypes = [C.c_void_p, P(C.c_double), P(C.c_int), C.c_int,
                                     P(C.c_double), P(C.c_int), C.c_int]
        L.orc_warm_start.argtypes = [C.c_void_p, P(C.c_double), P(C.c_double)]
        L.orc_solve.argtypes = [C.c_void_p]
        L.orc_get_solution.argtypes = [C.c_void_p, P(C.c_double), P(C.c_double),
                                       P(C.c_double), P(C.c_double)]
        L.orc_get_info.argtypes = [C.c_void_p, P(_Info)]
        L.orc_cleanup.argtypes = [C.c_void_p]
        L.orc_kkt_nnz_L.argtypes = [C.c_void_p]
        L.orc_solve_batch.argtypes = [C.c_int, C.c_int, C.c_int,
                                      P(C.c_int), P(C.c_int), P(C.c_double), P(C.c_double),
                                      P(C.c_int), P(C.c_int), P(C.c_double),
                                      P(C.c_double), P(C.c_double), P(_Settings),
                                      P(C.c_double), P(C.c_double), P(C.c_int), P(C.c_int),
                                      C.c_int]
        L.orc_solve_batch_warm.argtypes = [C.c_int, C.c_int, C.c_int,
                                           P(C.c_int), P(C.c_int), P(C.c_double), P(C.c_double),
                                           P(C.c_int), P(C.c_int), P(C.c_double),
                                           P(C.c_double), P(C.c_double), P(C.c_double), P(C.c_double),
                                           P(_Settings), P(C.c_double), P(C.c_double), P(C.c_int), P(C.c_int),
                                           C.c_int]
        L.orc_solve_batch_timed.argtypes = L.orc_solve_batch_warm.argtypes + [P(C.c_double)]
        _lib = L
    return _lib


def _dp(a):
    return None if a is None else a.ctypes.data_as(C.POINTER(C.c_double))


def _ip(a):
    return a.ctypes.data_as(C.POINTER(C.c_int))


_SETTING_KEYS = {f[0] for f in _Settings._fields_}


def make_settings(**kw) -> _Settings:
    s = _Settings()
    lib().orc_default_settings(C.byref(s))
    for k, v in kw.items():
        if k == "verbose":
            continue
        if k not in _SETTING_KEYS:
            raise ValueError(f"unknown setting {k}")
        setattr(s, k, type(getattr(s, k))(v))
    return s


def canon(P, A):
    """The osqp-python data canonicalisation: triu(P) CSC, A CSC, int32 indices."""
    P = sparse.triu(sparse.csc_matrix(P), format="csc")
    A = sparse.csc_matrix(A)
    P.sort_indices()
    A.sort_indices()
    return P, A


class OSQP:
    """Oracle with the osqp.OSQP surface (setup / update / warm_start / solve)."""

    def __init__(self):
        self._w = C.c_void_p()
        self.n = self.m = 0

    def setup(self, P, q, A, l, u, **settings):
        P, A = canon(P, A)
        self.n, self.m = P.shape[0], A.shape[0]
        s = make_settings(**settings)
        self._settings = dict(settings)
        self._keep = []
        arrs = [np.ascontiguousarray(P.indptr, np.int32), np.ascontiguousarray(P.indices, np.int32),
                np.ascontiguousarray(P.data, np.float64), np.ascontiguousarray(q, np.float64),
                np.ascontiguousarray(A.indptr, np.int32), np.ascontiguousarray(A.indices, np.int32),
                np.ascontiguousarray(A.data, np.float64), np.ascontiguousarray(l, np.float64),
                np.ascontiguousarray(u, np.float64)]
        e = lib().orc_setup(C.byref(self._w), self.n, self.m, _ip(arrs[0]), _ip(arrs[1]), _dp(arrs[2]),
                            _dp(arrs[3]), _ip(arrs[4]), _ip(arrs[5]), _dp(arrs[6]), _dp(arrs[7]),
                            _dp(arrs[8]), C.byref(s))
        if e:
            raise ValueError(f"oracle setup failed (code {e})")

    def update(self, q=None, l=None, u=None, Px=None, Px_idx=None, Ax=None, Ax_idx=None):
        """osqp.OSQP.update in osqp-python 0.6's order: q, the bounds, then the matrices
        (update_P / update_A / update_P_A; an empty or missing index array: all values)."""
        L = lib()
        e = 0
        if q is not None:
            q = np.ascontiguousarray(q, np.float64)
            L.orc_update_lin_cost(self._w, _dp(q))
        if l is not None and u is not None:
            l = np.ascontiguousarray(l, np.float64); u = np.ascontiguousarray(u, np.float64)
            e = L.orc_update_bounds(self._w, _dp(l), _dp(u))
        elif l is not None:
            l = np.ascontiguousarray(l, np.float64)
            e = L.orc_update_lower_bound(self._w, _dp(l))
        elif u is not None:
            u = np.ascontiguousarray(u, np.float64)
            e = L.orc_update_upper_bound(self._w, _dp(u))
        if e:
            raise ValueError(f"oracle update failed (code {e})")
        if Px is not None or Ax is not None:
            def prep(v, idx):
                if v is None:
                    return None, None, 0
                v = np.ascontiguousarray(v, np.float64)
                if idx is None or np.size(idx) == 0:
                    return v, None, v.size
                return v, np.ascontiguousarray(idx, np.int32), v.size
            Pv, Pi, nP = prep(Px, Px_idx)
            Av, Ai, nA = prep(Ax, Ax_idx)
            e = L.orc_update_P_A(self._w, _dp(Pv), None if Pi is None else _ip(Pi), nP,
                                 _dp(Av), None if Ai is None else _ip(Ai), nA)
            if e:
                raise ValueError(f"oracle matrix update failed (code {e})")

    def update_settings(self, **kw):
        """osqp.OSQP.update_settings: the settings OSQP lets change after setup"""
        new = dict(self._settings, **kw)
        s = make_settings(**new)
        e = lib().orc_update_settings(self._w, C.byref(s), int("rho" in kw))
        if e:
            raise ValueError(f"oracle update_settings failed (code {e})")
        self._settings = new

    def warm_start(self, x=None, y=None):
        x = np.ascontiguousarray(x, np.float64); y = np.ascontiguousarray(y, np.float64)
        lib().orc_warm_start(self._w, _dp(x), _dp(y))
        self._settings["warm_start"] = True  # (osqp_warm_start turns the setting on)

    def solve(self):
        L = lib()
        L.orc_solve(self._w)
        x = np.empty(self.n); y = np.empty(self.m)
        pc = np.empty(self.m); dc = np.empty(self.n)
        L.orc_get_solution(self._w, _dp(x), _dp(y), _dp(pc), _dp(dc))
        info = _Info()
        L.orc_get_info(self._w, C.byref(info))
        inf = SimpleNamespace(iter=info.iter, status_val=info.status_val,
                              status=STATUS_STR.get(info.status_val, "unknown"),
                              obj_val=info.obj_val, pri_res=info.pri_res, dua_res=info.dua_res,
                              rho_estimate=info.rho_estimate, rho_updates=info.rho_updates,
                              status_polish=info.status_polish)
        return SimpleNamespace(x=x, y=y, info=inf, prim_inf_cert=pc, dual_inf_cert=dc)

    def nnz_L(self):
        return lib().orc_kkt_nnz_L(self._w)

    def __del__(self):
        if getattr(self, "_w", None) and self._w.value and lib is not None:  # module torn down at exit
            lib().orc_cleanup(self._w)
            self._w = C.c_void_p()


def solve_batch(P, A, Px_b, q_b, Ax_b, l_b, u_b, nthreads=1, x0=None, y0=None, **settings):
    """B fresh setup()+solve() runs with a shared pattern (values per instance);
    with x0 (B, n) and y0 (B, m) each instance is warm-started after its setup."""
    P, A = canon(P, A)
    n, m = P.shape[0], A.shape[0]
    B = q_b.shape[0]
    s = make_settings(**settings)
    Pp = np.ascontiguousarray(P.indptr, np.int32); Pi = np.ascontiguousarray(P.indices, np.int32)
    Ap = np.ascontiguousarray(A.indptr, np.int32); Ai = np.ascontiguousarray(A.indices, np.int32)
    Px_b = np.ascontiguousarray(Px_b, np.float64); Ax_b = np.ascontiguousarray(Ax_b, np.float64)
    q_b = np.ascontiguousarray(q_b, np.float64)
    l_b = np.ascontiguousarray(l_b, np.float64); u_b = np.ascontiguousarray(u_b, np.float64)
    x = np.empty((B, n)); y = np.empty((B, m))
    st = np.empty(B, np.int32); it = np.empty(B, np.int32)
    if (x0 is None) != (y0 is None):
        raise ValueError("x0 and y0 go together")
    if x0 is not None:
        x0 = np.ascontiguousarray(x0, np.float64); y0 = np.ascontiguousarray(y0, np.float64)
    ph = np.zeros(2)
    e = lib().orc_solve_batch_timed(B, n, m, _ip(Pp), _ip(Pi), _dp(Px_b), _dp(q_b), _ip(Ap), _ip(Ai),
                                    _dp(Ax_b), _dp(l_b), _dp(u_b), _dp(x0), _dp(y0), C.byref(s), _dp(x),
                                    _dp(y), _ip(st), _ip(it), int(nthreads), _dp(ph))
    # t_setup / t_solve: thread-seconds in setup (+ warm start) and in solve
    return SimpleNamespace(x=x, y=y, status_val=st, iter=it, err=e, t_setup=float(ph[0]), t_solve=float(ph[1]))
