#!/usr/bin/env python3
"""Diagnostic (GPU): max |x - x_oracle| after k iterations (max_iter = k) on a small cfg-2
batch, for the mode MPCQP_DENSE_W4 selects -- where a kernel form's iterates leave the
oracle's."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.environ.get("MPCQP_PKG", os.path.join(ROOT, "python-mpc_amd")), os.path.join(ROOT, "oracle")]
import pyoracle  # noqa: E402
from osqp_amd import OSQPBatch, mpc  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
b = mpc.make_batch(2, B=B)
for ct in (0, 1):
    for k in (1, 2, 3, 4, 8, 25, 26, 50):
        settings = {"max_iter": k, "check_termination": ct, "adaptive_rho": False}
        bo = pyoracle.solve_batch(b["P"], b["A"], b["Px"], b["q"], b["Ax"], b["l"], b["u"], nthreads=8, **settings)
        bg = OSQPBatch()
        bg.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **settings)
        rg = bg.solve()
        dx = np.abs(rg.x - bo.x).max(axis=1)
        dy = np.abs(rg.y - bo.y).max(axis=1)
        print(f"check {ct} max_iter {k:3d}: max|dx| {np.nanmax(dx):.3e} max|dy| {np.nanmax(dy):.3e} "
              f"status {rg.status_val[:4]} {bo.status_val[:4]} argmax col {int(np.nanargmax(np.abs(rg.x - bo.x).max(axis=0)))}")
