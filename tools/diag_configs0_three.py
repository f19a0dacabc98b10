#!/usr/bin/env python3
"""configs[0] loop, steps 1000-1100 (the stretch where the device and the oracle part;
tests/test_gpu_parity.py::test_slack_script_configs0_1500_steps): three solvers on the same
step QPs from the same start.  The oracle runs the script's 1500-step loop and records each
step's QP (q, l, u as solved) and its solution; then for every step s of the window all
three solvers solve QP_s warm-started from the oracle's solution of step s-1 (osqp_warm_start:
x, y, z = A x) -- so each step is compared from an identical start, free of the warm-start
drift of a driven loop:
  oracle  oracle/osqp_oracle.c (quasi-definite LDL', OSQP 0.6's KKT form)
  dense   tests/osqp_dense_ref.py (numpy, explicit inverse of P + sigma I + A' rho A)
  device  the MI355X solver (the reduced form through the block inverse), one batch
Prints each step where the iteration counts differ and which solver is the odd one out.

  python tools/diag_configs0_three.py [--lo 1000 --hi 1100]   (GPU)
  python tools/diag_configs0_three.py --loops   (GPU): the loops themselves, below
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("tests", "python-mpc_amd", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np  # noqa: E402
import pyoracle  # noqa: E402
import osqp_dense_ref  # noqa: E402
from osqp_amd import OSQPBatch, mpc  # noqa: E402


def record(nsim, N=20):
    """The script's loop with the oracle (test_gpu_parity._slack_script_loop's calls),
    recording each step's solved (q, l, u) and the solution."""
    x0 = np.array([0.0, 0.0, 5 * mpc.DEG, 3.0, 0.0])
    P, q, A, l, u = mpc.slack_qp(N, x0)
    o = pyoracle.OSQP()
    o.setup(P, q, A, l, u, warm_start=True)
    At, Bt = mpc.augment(mpc.LATERAL_AD, mpc.LATERAL_BD)
    nx = At.shape[0]
    cur_l, cur_u = l.copy(), u.copy()
    Q, L, U, X, Y, IT = [], [], [], [], [], []
    for i in range(nsim):
        regime = 0 if i <= 400 else (1 if i <= 900 else 0)
        _, q_new, _, l_new, u_new = mpc.slack_qp(N, x0, regime=regime)
        o.update(q=q_new, l=l_new, u=u_new)
        r = o.solve()
        Q.append(q_new.copy()); L.append(l_new.copy()); U.append(u_new.copy())
        X.append(r.x.copy()); Y.append(r.y.copy()); IT.append(r.info.iter)
        d = r.x[(N + 1) * nx:(N + 1) * nx + 1]
        x0 = At @ x0 + Bt @ d
        l_new[:nx] = -x0
        u_new[:nx] = -x0
        o.update(l=l_new, u=u_new)
    return P, A, np.array(Q), np.array(L), np.array(U), np.array(X), np.array(Y), np.array(IT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lo", type=int, default=1000)
    ap.add_argument("--hi", type=int, default=1100)
    a = ap.parse_args()
    P, A, Q, L, U, X, Y, IT = record(a.hi + 1)
    if os.environ.get("DIAG_CPU_ONLY") == "1":  # (the oracle / dense part alone, no device)
        globals()["OSQPBatch"] = None
    steps = np.arange(a.lo, a.hi + 1)
    Pd, Ad = P.toarray(), A.toarray()
    it_o, it_d, it_g = [], [], []
    xs_o, xs_d = [], []
    # oracle and dense, one step at a time from the oracle's previous solution
    for s in steps:
        o = pyoracle.OSQP()
        o.setup(P, Q[s], A, L[s], U[s], warm_start=True)
        o.warm_start(x=X[s - 1], y=Y[s - 1])
        ro = o.solve()
        it_o.append(ro.info.iter)
        xs_o.append(ro.x.copy())
        xd, _, st, k, _ = osqp_dense_ref.solve(Pd, Q[s], Ad, L[s], U[s], x0=X[s - 1], y0=Y[s - 1])
        it_d.append(k)
        xs_d.append(xd)
    # the device: the window as one batch, each instance warm-started the same way
    B = len(steps)
    if OSQPBatch is None:
        it_o, it_d = np.array(it_o), np.array(it_d)
        print(f"oracle == dense at {np.sum(it_o == it_d)} of {B}:", [(int(s), int(i), int(j)) for s, i, j in zip(steps, it_o, it_d) if i != j])
        return
    g = OSQPBatch()
    g.setup(P, Q[steps], A, L[steps], U[steps], warm_start=True)
    g.warm_start(x=X[steps - 1], y=Y[steps - 1])
    r = g.solve()
    it_g = list(np.asarray(r.iter))
    it_o, it_d, it_g = np.array(it_o), np.array(it_d), np.array(it_g)
    xs_o, xs_d = np.array(xs_o), np.array(xs_d)
    same = (it_o == it_d) & (it_o == it_g)
    scale = np.maximum(1.0, np.abs(xs_o).max(axis=1))
    e_d = (np.abs(xs_d - xs_o).max(axis=1) / scale)[same]
    e_g = (np.abs(np.asarray(r.x) - xs_o).max(axis=1) / scale)[same]
    N, nx = 20, 5  # the augmented lateral state (mpc.augment: 4 + 1)
    j = (N + 1) * nx
    u_d = np.abs(xs_d[:, j] - xs_o[:, j])[same]
    u_g = np.abs(np.asarray(r.x)[:, j] - xs_o[:, j])[same]
    q = lambda v: f"median {np.median(v):.1e}, p90 {np.quantile(v, 0.9):.1e}, max {v.max():.1e}"  # noqa: E731
    print(f"  where all three agree on the count: |x - x_oracle|_inf / max(1, |x|_inf): dense {q(e_d)}; device {q(e_g)}")
    print(f"                                      |du_0 - du_0 oracle|: dense {q(u_d)}; device {q(u_g)}")
    print(f"steps {a.lo}..{a.hi}, each from the oracle's previous solution (x, y; z = A x)")
    print(f"  oracle == dense  at {np.sum(it_o == it_d)} of {B} steps")
    print(f"  oracle == device at {np.sum(it_o == it_g)} of {B} steps")
    print(f"  dense  == device at {np.sum(it_d == it_g)} of {B} steps")
    print(f"  the loop's own (drifting warm start) oracle counts at these steps: {IT[steps].tolist()[:12]} ...")
    for k, s in enumerate(steps):
        if not (it_o[k] == it_d[k] == it_g[k]):
            odd = "oracle" if it_d[k] == it_g[k] else ("dense" if it_o[k] == it_g[k] else
                                                      ("device" if it_o[k] == it_d[k] else "all differ"))
            print(f"  step {s}: oracle {it_o[k]}, dense {it_d[k]}, device {it_g[k]}  -> odd one out: {odd}")


if __name__ == "__main__" and "--loops" not in sys.argv:
    main()


def loops():
    """The script's loop as the GPU test runs it, three solvers: each warm-starts from its own
    solutions, driven along the oracle's plant states; then each free-running."""
    from test_gpu_parity import _slack_script_loop
    import importlib.util
    spec = importlib.util.spec_from_file_location("osqp", os.path.join(ROOT, "python-mpc_amd", "shim", "osqp.py"))
    shim = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(shim)
    log = []

    class Dense(osqp_dense_ref.OSQP):
        def solve(self):
            r = super().solve()
            log.append(self.last_checks)
            return r
    dense = type("m", (), {"OSQP": Dense})
    o, xo = _slack_script_loop(pyoracle)
    d, _ = _slack_script_loop(dense, states=xo)
    g, _ = _slack_script_loop(shim, states=xo)
    print("driven along the oracle's plant states (each solver warm-starts from its own solutions):")
    for tag, r in (("dense", d), ("device", g)):
        mm = np.flatnonzero(r[:, 1] != o[:, 1])
        du = np.abs(r[:, 0] - o[:, 0])
        print(f"  {tag}: iteration counts differ from the oracle's at {mm.size} steps {mm.tolist()[:20]}; "
              f"du_0 max diff {du[:800].max():.2e} (steps < 800), {du[:1000].max():.2e} (< 1000), {du.max():.2e} (all)")
    for s in np.flatnonzero(g[:, 1] != o[:, 1]):
        k = int(min(g[s, 1], o[s, 1]))
        ratio = dict(log[s]).get(k, float("nan"))
        print(f"    step {s}: device {int(g[s, 1])}, oracle {int(o[s, 1])}, dense {int(d[s, 1])}; at check {k} the "
              f"dense chain's max(prim/eps_prim, dual/eps_dual) = {ratio:.5f} (decision margin {abs(ratio - 1):.2%})")
    log.clear()
    df, xd = _slack_script_loop(dense)
    gf, xg = _slack_script_loop(shim)
    print("free-running (each on its own plant trajectory):")
    for tag, r, xs in (("dense", df, xd), ("device", gf, xg)):
        du = np.abs(r[:, 0] - o[:, 0])
        mm = np.flatnonzero(r[:, 1] != o[:, 1])
        first = int(np.argmax(du > 1e-4)) if np.any(du > 1e-4) else None
        print(f"  {tag}: du_0 max diff {du[:800].max():.2e} (steps < 800), {du[:1000].max():.2e} (< 1000), "
              f"first step > 1e-4: {first}; iteration mismatches {mm.size} (first {mm[:3].tolist()}); "
              f"max |x| per state {np.abs(xs).max(0).round(3).tolist()} vs oracle {np.abs(xo).max(0).round(3).tolist()}")


if __name__ == "__main__" and "--loops" in sys.argv:
    loops()
