#!/usr/bin/env python3
"""Diagnostic (GPU only): compare solve-kernel variants iterate by iterate.

Runs the same seeded batch with a fixed number of ADMM iterations (no
termination checks, no rho adaptation) under two MPCQP_VARIANT values and
prints the largest difference of x after k iterations -- an exact linear solve
in both variants keeps it at rounding level for every k.

  python tools/variant_diff.py --config 2 --variants 0 8
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-mpc_amd"))

import numpy as np  # noqa: E402


def run(variant, b, iters, B, adaptive):
    os.environ["MPCQP_VARIANT"] = str(variant)
    from osqp_amd import OSQPBatch
    s = OSQPBatch()
    s.setup(P=b["P"], q=b["q"], A=b["A"], l=b["l"], u=b["u"], Px=b["Px"], Ax=b["Ax"],
            eps_abs=0.0, eps_rel=1e-300, eps_prim_inf=1e-300, eps_dual_inf=1e-300,
            adaptive_rho=adaptive, max_iter=iters, check_termination=0, warm_start=False)
    r = s.solve()
    return r.x


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--variants", type=int, nargs=2, default=[0, 8])
    ap.add_argument("--iters", type=int, nargs="+", default=[1, 2, 3, 5, 10, 25, 50, 100])
    a = ap.parse_args()
    from osqp_amd import mpc
    b = mpc.make_batch(a.config, B=a.batch, seed=7)
    for it in a.iters:
        x0 = run(a.variants[0], b, it, a.batch, False)
        x1 = run(a.variants[1], b, it, a.batch, False)
        d = np.abs(x0 - x1).max()
        print(f"iters {it:4d}: max |x_v{a.variants[0]} - x_v{a.variants[1]}| = {d:.3e}  (|x| {np.abs(x0).max():.3e})",
              flush=True)


if __name__ == "__main__":
    main()
