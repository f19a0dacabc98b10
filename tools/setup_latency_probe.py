#!/usr/bin/env python3
"""Where a small setup's time goes (GPU only, diagnostic): osqp-python's data
canonicalisation, mpcqp_setup_batch + mpcqp_free, mpcqp_create + mpcqp_free (allocation
only), and the shim's whole OSQP().setup(), in microseconds per call, on one QP of the
given config (default 2).

  python tools/setup_latency_probe.py [config]
"""
import sys, time, os
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "python-mpc_amd"))
import ctypes as C
import numpy as np
import osqp_amd as oa
from osqp_amd import mpc, lib, _make_settings, canonical_data, _dp, _ip
cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
b = mpc.make_batch(cfg, B=1, seed=1)
P, A = b["P"].copy(), b["A"].copy(); P.data, A.data = b["Px"][0].copy(), b["Ax"][0].copy()
q, l, u = b["q"][0].copy(), b["l"][0].copy(), b["u"][0].copy()
L = lib()
Pc, Ac = canonical_data(P, A)
Pp, Pi, Ap, Ai = (np.ascontiguousarray(v, np.int32) for v in (Pc.indptr, Pc.indices, Ac.indptr, Ac.indices))
Px, Ax = np.ascontiguousarray(Pc.data[None, :]), np.ascontiguousarray(Ac.data[None, :])
qq, ll, uu = q[None, :].copy(), l[None, :].copy(), u[None, :].copy()
s = _make_settings(warm_start=True)
nn, mm = P.shape[0], A.shape[0]
def t(f, k=30):
    f()
    t0 = time.perf_counter()
    for _ in range(k): f()
    return (time.perf_counter() - t0) / k * 1e6
def c_setup():
    h = C.c_void_p()
    L.mpcqp_setup_batch(nn, mm, _ip(Pp), _ip(Pi), _ip(Ap), _ip(Ai), 1, _dp(Px), _dp(Ax), _dp(qq), _dp(ll), _dp(uu), C.byref(s), 1, C.byref(h))
    L.mpcqp_free(h)
def c_create():
    h = C.c_void_p()
    L.mpcqp_create(nn, mm, _ip(Pp), _ip(Pi), _ip(Ap), _ip(Ai), 1, C.byref(s), 0, C.byref(h))
    L.mpcqp_free(h)
def py_setup():
    o = oa.OSQP(); o.setup(P, q, A, l, u, warm_start=True, verbose=False)
def canon():
    canonical_data(P, A)
print("config", cfg, "n", nn, "m", mm)
print("canonical_data us", t(canon))
print("C setup_batch+free us", t(c_setup))
print("C create+free us", t(c_create))
print("OSQP().setup (+free at gc) us", t(py_setup))
