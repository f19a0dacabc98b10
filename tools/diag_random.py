#!/usr/bin/env python3
"""Diagnostic (GPU): the random banded batches of tests/test_gpu_parity.py, instance by
instance.  For every instance where the device and the oracle differ in status, iteration
count or NaN-ness it prints the three solvers side by side -- the device (reduced SPD
system P + sigma I + A' rho A, block LDL'), the oracle (quasi-definite KKT, LDL' with a
minimum-degree ordering, as OSQP's QDLDL) and tests/osqp_dense_ref.py (the reduced system
again, explicitly inverted by LAPACK) -- with the conditioning of the two linear systems at
the first factorisation (scaled data, rho0): cond of the reduced matrix, of the
quasi-definite KKT matrix, and the ratio.  Then the largest |x - x_ref| among instances
with equal iteration counts."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "python-mpc_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

spec = importlib.util.spec_from_file_location("t", os.path.join(ROOT, "tests", "test_gpu_parity.py"))
t = importlib.util.module_from_spec(spec)
spec.loader.exec_module(t)
import osqp_dense_ref  # noqa: E402
import pyoracle  # noqa: E402
from osqp_amd import OSQPBatch  # noqa: E402

ST = {1: "solved", -3: "prim_inf", -2: "max_it", 2: "solved_inacc", -4: "dual_inf", -7: "non_cvx"}


def conds(P, A, l, u, sigma=1e-6, rho=0.1):
    """cond of the reduced and the quasi-definite KKT matrices after OSQP's Ruiz scaling
    (the dense restatement's scaling loop), at rho0 with OSQP's rho classes."""
    Pd = np.triu(P.toarray()); Ad = A.toarray()
    n, m = Pd.shape[0], Ad.shape[0]
    Pf = lambda Pu: Pu + np.triu(Pu, 1).T
    lim = lambda v: np.where(v < 1e-4, 1.0, np.where(v > 1e4, 1e4, v))
    for _ in range(10):
        Dt = 1 / np.sqrt(lim(np.maximum(np.abs(Pf(Pd)).max(0), np.abs(Ad).max(0))))
        Et = 1 / np.sqrt(lim(np.abs(Ad).max(1)))
        Pd = Dt[:, None] * Pd * Dt[None, :]; Ad = Et[:, None] * Ad * Dt[None, :]
        l = Et * l; u = Et * u
    r = np.where(u - l < 1e-4, 1e3 * rho, rho)
    r = np.where((l < -1e26) & (u > 1e26), 1e-6, r)
    Kr = Pf(Pd) + sigma * np.eye(n) + Ad.T @ (r[:, None] * Ad)
    Kq = np.block([[Pf(Pd) + sigma * np.eye(n), Ad.T], [Ad, -np.diag(1 / r)]])
    cr, cq = np.linalg.cond(Kr), np.linalg.cond(Kq)
    return cr, cq


def main():
    s = dict(warm_start=False, polish=False)
    for case in [(60, 40, 2, 1), (150, 90, 3, 2), (300, 200, 1, 3)]:
        b = t._random_banded_batch(96, *case)
        bo = pyoracle.solve_batch(b["P"], b["A"], b["Px"], b["q"], b["Ax"], b["l"], b["u"], nthreads=16, **s)
        bg = OSQPBatch()
        bg.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
        rg = bg.solve()
        info = bg.plan_info()
        print(f"case n={case[0]} m={case[1]} band={case[2]} seed={case[3]}: variant {info['variant']}, nb {info['nb']}; "
              f"statuses device {dict(zip(*np.unique(rg.status_val, return_counts=True)))} "
              f"oracle {dict(zip(*np.unique(bo.status_val, return_counts=True)))}", flush=True)
        P, A = b["P"].copy(), b["A"].copy()
        bad = 0
        for k in range(96):
            gn, on = np.isnan(rg.x[k]).sum(), np.isnan(bo.x[k]).sum()
            if rg.iter[k] == bo.iter[k] and rg.status_val[k] == bo.status_val[k] and gn == on:
                continue
            bad += 1
            P.data, A.data = b["Px"][k], b["Ax"][k]
            xd, yd, std, itd, _ = osqp_dense_ref.solve(P.toarray(), b["q"][k], A.toarray(), b["l"][k], b["u"][k])
            cr, cq = conds(P, A, b["l"][k], b["u"][k])
            print(f"  k={k:2d} device {ST.get(int(rg.status_val[k]), rg.status_val[k])}/{rg.iter[k]} nan={gn} | "
                  f"oracle {ST.get(int(bo.status_val[k]), bo.status_val[k])}/{bo.iter[k]} nan={on} | "
                  f"dense-reduced {std}/{itd} | cond reduced {cr:.2e} quasi-definite {cq:.2e} ratio {cr / cq:.2e}",
                  flush=True)
        ok = np.isfinite(bo.x).all(axis=1) & (rg.iter == bo.iter) & (rg.status_val == bo.status_val)
        du = np.abs(rg.x - bo.x).max(axis=1)
        print(f"  mismatches {bad}/96; equal status+iterations: {ok.sum()}, of them max |x - x_ref| "
              f"{du[ok].max():.2e}, median {np.median(du[ok]):.2e}", flush=True)


if __name__ == "__main__":
    main()
