#!/usr/bin/env python3
"""Diagnostic (GPU): the four-wave kernel's dense-inverse form against the oracle on a small
cfg-2 batch -- statuses, iteration counts, max |x - x_oracle| -- for the mode MPCQP_DENSE_W4 /
MPCQP_BALANCE select (run once per mode in separate processes).

  MPCQP_DENSE_W4=1 python tools/diag_dense.py [B]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.environ.get("MPCQP_PKG", os.path.join(ROOT, "python-mpc_amd")), os.path.join(ROOT, "oracle")]
import pyoracle  # noqa: E402
from osqp_amd import OSQPBatch, mpc  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
cfg = int(sys.argv[2]) if len(sys.argv) > 2 else 2
b = mpc.make_batch(cfg, B=B)
for settings in ({}, {"max_iter": 1, "check_termination": 1}, {"max_iter": 25, "check_termination": 25}):
    bo = pyoracle.solve_batch(b["P"], b["A"], b["Px"], b["q"], b["Ax"], b["l"], b["u"], nthreads=8, **settings)
    bg = OSQPBatch()
    bg.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **settings)
    print("plan", {k: v for k, v in bg.plan_info().items() if k in ("nb", "amax", "variant", "npad")})
    rg = bg.solve()
    dx = np.abs(rg.x - bo.x).max(axis=1)
    print(settings, "status", rg.status_val[:8], bo.status_val[:8], "iter", rg.iter[:8], bo.iter[:8],
          "max|dx|", np.nanmax(dx), "nan", int(np.isnan(rg.x).any(axis=1).sum()))
    print("  x[0,:8]", rg.x[0, :8], "\n  oracle ", bo.x[0, :8])
