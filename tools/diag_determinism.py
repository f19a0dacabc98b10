#!/usr/bin/env python3
"""Diagnostic (GPU): solve the same cfg-2 batch several times on fresh handles (host API,
setup + solve kernels) and once through the fused device path; report whether the
outputs are bitwise identical across runs and the worst |u - u_oracle|."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "python-mpc_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
import pyoracle  # noqa: E402
from osqp_amd import OSQPBatch, mpc  # noqa: E402

b = mpc.make_batch(2, B=1024)
s = dict(warm_start=True)
bo = pyoracle.solve_batch(b["P"], b["A"], b["Px"], b["q"], b["Ax"], b["l"], b["u"], nthreads=16, **s)
runs = []
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
    bg = OSQPBatch()
    bg.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
    rg = bg.solve()
    runs.append(rg)
    du = np.abs(rg.x[:, b["u_block"]] - bo.x[:, b["u_block"]]).max(axis=1)
    same = rg.iter == bo.iter
    k = int(np.argmax(np.where(same, du, -1)))
    print(f"run {rep}: iter match {same.mean():.4f} worst du (same iters) {du[same].max():.3e} at {k} "
          f"(iters {rg.iter[k]}), status match {(rg.status_val == bo.status_val).mean():.4f}", flush=True)
for rep in range(1, len(runs)):
    dx = np.abs(runs[rep].x - runs[0].x).max(axis=1)
    bad = np.flatnonzero(dx != 0)
    print(f"run {rep} vs 0: {bad.size} instances differ; first {bad[:8].tolist()} max {dx.max():.3e}; "
          f"iters differ {np.flatnonzero(runs[rep].iter != runs[0].iter)[:8].tolist()}")
