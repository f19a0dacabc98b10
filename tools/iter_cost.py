#!/usr/bin/env python3
"""Per-ADMM-iteration cost of k_solve, measured without in-kernel stamps (GPU only).

All instances are forced to run exactly max_iter iterations (eps = 0, no
infeasibility exit, adaptive rho off, termination checks every `--check`
iterations or never), and the kernel time is measured at two max_iter values:
the slope is the cost of one iteration of the whole batch in lock step, the
intercept the setup + factorisation + epilogue.

  python tools/iter_cost.py --config 2 [--variant 7] [--check 25]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-mpc_amd"))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--variant", type=int, default=None)
    ap.add_argument("--check", type=int, default=0, help="check_termination (0: never)")
    ap.add_argument("--iters", type=int, nargs=2, default=[50, 250])
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    if a.variant is not None:
        os.environ["MPCQP_VARIANT"] = str(a.variant)
    import torch
    from osqp_amd import DeviceBatch, mpc, _drop_common_zeros
    spec = mpc.CONFIGS[a.config]
    B = a.batch or spec["B"]
    b = mpc.make_batch(a.config, B=B, seed=7)
    P, Px = _drop_common_zeros(b["P"], b["Px"])
    A, Ax = _drop_common_zeros(b["A"], b["Ax"])
    dev = torch.device("cuda", 0)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
    dPx, dAx, dq, dl, du = (t(x) for x in (Px, Ax, b["q"], b["l"], b["u"]))
    dx = torch.empty((B, b["n"]), dtype=torch.float64, device=dev)
    dy = torch.empty((B, b["m"]), dtype=torch.float64, device=dev)
    dst = torch.empty(B, dtype=torch.int32, device=dev)
    dit = torch.empty(B, dtype=torch.int32, device=dev)
    res = []
    for it in a.iters:
        s = DeviceBatch(P, A, B, device=0, eps_abs=0.0, eps_rel=1e-300, eps_prim_inf=1e-300, eps_dual_inf=1e-300,
                        adaptive_rho=False, max_iter=it, check_termination=a.check, warm_start=False)
        for _ in range(2):
            s.setup(dPx, dAx, dq, dl, du)
            s.solve(dx, dy, dst, dit)
        s.synchronize()
        s.timing(True)
        for _ in range(a.reps):
            s.setup(dPx, dAx, dq, dl, du)
            s.solve(dx, dy, dst, dit)
        kt = s.timing_read()
        s.timing(False)
        its = dit.cpu().numpy()
        assert (its == it).all(), (its.min(), its.max())
        res.append(kt["solve_ms"] / kt["n_solve"])
        info = s.plan_info()
        del s
    (i0, i1), (t0, t1) = a.iters, res
    per_it = (t1 - t0) / (i1 - i0) * 1e3
    print(f"config {a.config} B={B} variant={os.environ.get('MPCQP_VARIANT', 'auto')} check={a.check} "
          f"lds={info['lds_bytes_solve']}: kernel {t0:.3f} ms @ {i0} it, {t1:.3f} ms @ {i1} it -> "
          f"{per_it:.3f} us/iteration (~{per_it * 2.4e3:.0f} cycles at 2.4 GHz), "
          f"intercept {t0 - per_it * i0 / 1e3:.3f} ms")


if __name__ == "__main__":
    main()
