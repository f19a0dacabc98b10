#!/usr/bin/env python3
"""Per-call latency of the `import osqp` shim on one QP (GPU only, diagnostic).

The reference's closed loop (vehicle_lateral_mpc_slack_increment.py:237,248) calls
update(q=, l=, u=) then solve() on ONE problem per control step; this times both calls on the
slack layout at N = 20 (configs[0]) and prints the mean and median microseconds per call,
then a fresh object's setup() + solve() per call (the Control/MPC scripts' pattern).

  python tools/shim_latency.py [--steps 300]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-mpc_amd"))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--config", type=int, default=3)
    a = ap.parse_args()
    from osqp_amd import OSQP, mpc
    b = mpc.make_batch(a.config, B=1, seed=1)
    P, A = b["P"].copy(), b["A"].copy()
    P.data, A.data = b["Px"][0].copy(), b["Ax"][0].copy()
    q, l, u = b["q"][0].copy(), b["l"][0].copy(), b["u"][0].copy()
    prob = OSQP()
    prob.setup(P, q, A, l, u, warm_start=True, verbose=False)
    for _ in range(20):
        prob.update(q=q, l=l, u=u)
        prob.solve()
    tu, ts, its = [], [], []
    for _ in range(a.steps):
        t0 = time.perf_counter()
        prob.update(q=q, l=l, u=u)
        t1 = time.perf_counter()
        r = prob.solve()
        t2 = time.perf_counter()
        tu.append(t1 - t0)
        ts.append(t2 - t1)
        its.append(r.info.iter)
    f = lambda v: f"mean {1e6 * np.mean(v):.0f} us, median {1e6 * np.median(v):.0f} us"  # noqa: E731
    print(f"config {a.config}, one QP, warm: update(q,l,u) {f(tu)}; solve() {f(ts)}; iterations {np.mean(its):.0f}")
    # a fresh object per call (Control/MPC/mpc_kinematics.py:194-198: setup + solve every step)
    tsu, tso = [], []
    for _ in range(max(10, a.steps // 6)):
        t0 = time.perf_counter()
        p2 = OSQP()
        p2.setup(P, q, A, l, u, warm_start=True, verbose=False)
        t1 = time.perf_counter()
        p2.solve()
        t2 = time.perf_counter()
        tsu.append(t1 - t0)
        tso.append(t2 - t1)
    print(f"config {a.config}, fresh object per call: setup() {f(tsu)}; solve() {f(tso)}")


if __name__ == "__main__":
    main()
