#!/usr/bin/env python3
"""Diagnostic (GPU): the random banded batches of tests/test_gpu_parity.py, instance by
instance -- status / iterations / NaNs of the device solve against the oracle."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "python-mpc_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

spec = importlib.util.spec_from_file_location("t", os.path.join(ROOT, "tests", "test_gpu_parity.py"))
t = importlib.util.module_from_spec(spec)
spec.loader.exec_module(t)
import pyoracle  # noqa: E402
from osqp_amd import OSQPBatch  # noqa: E402

for case in [(60, 40, 2, 1), (150, 90, 3, 2), (300, 200, 1, 3)]:
    b = t._random_banded_batch(96, *case)
    s = dict(warm_start=False, polish=False)
    bo = pyoracle.solve_batch(b["P"], b["A"], b["Px"], b["q"], b["Ax"], b["l"], b["u"], nthreads=16, **s)
    bg = OSQPBatch()
    bg.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
    rg = bg.solve()
    print(case, "variant", bg.plan_info() if hasattr(bg, "plan_info") else "")
    for k in range(96):
        gn, on = np.isnan(rg.x[k]).sum(), np.isnan(bo.x[k]).sum()
        if rg.iter[k] != bo.iter[k] or rg.status_val[k] != bo.status_val[k] or gn != on:
            print(f"  k={k} gpu st={rg.status_val[k]} it={rg.iter[k]} nan={gn} | oracle st={bo.status_val[k]} "
                  f"it={bo.iter[k]} nan={on} | ynan gpu={np.isnan(rg.y[k]).sum()} orc={np.isnan(bo.y[k]).sum()}")
    ok = np.isfinite(bo.x).all(axis=1) & (rg.iter == bo.iter)
    du = np.abs(rg.x - bo.x).max(axis=1)
    worst = np.argsort(np.where(ok, du, -1))[::-1][:5]
    print("  statuses", np.unique(rg.status_val, return_counts=True))
    print("  worst |x - x_ref| (same iterations):", [(int(k), float(du[k]), int(rg.iter[k]), int(rg.status_val[k])) for k in worst])
