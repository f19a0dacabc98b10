"""BASELINE.json's full-size slack workload (configs[2]: 65536 QPs), every instance checked.

The oracle finishes a few hundred of these instances in seconds, not 65536, so at full size
the check is a size-independent property: each returned (x, y) must satisfy OSQP's own
termination test for status "solved" (OSQP 0.6 check_termination, unscaled residuals):

  dual:   ||P x + q + A'y||_inf <= eps_abs + eps_rel * max(||P x||, ||A'y||, ||q||)
  primal: dist(A x, [l, u])_inf <= ||A x - z||_inf <= eps_abs + eps_rel * max(||A x||, ||z||),
          and with ||z|| <= ||A x|| + ||A x - z||:  dist <= (eps_abs + eps_rel ||A x||) / (1 - eps_rel)

computed on the host from the instance's CSC values with numpy, for the first solve and for
a second solve of moved initial states, which the kernel dispatches longest-previous-first
(the order the timed bench steps run in).  The oracle pins a sample of the same batch.
"""
import numpy as np
import pytest

import pyoracle
from osqp_amd import OSQPBatch, mpc

pytestmark = pytest.mark.gpu  # (the checker itself is CPU-tested: test_fullsize_checker.py)

EPS = 1e-3
SLACK = 1e-9  # host recomputation of the residuals (fp64 sums in another order)


def _csc_rows_cols(M):
    cols = np.repeat(np.arange(M.shape[1]), np.diff(M.indptr))
    return M.indices.astype(np.int64), cols


def _matvec(rows, cols, vals, x, nrow):
    """Batched y[b] = M_b x[b] for one CSC pattern with per-instance values (B, nnz):
    the products grouped by row and summed with one reduceat over the batch."""
    order = np.argsort(rows, kind="stable")
    r = rows[order]
    contrib = vals[:, order] * x[:, cols[order]]
    starts = np.flatnonzero(np.r_[True, r[1:] != r[:-1]]) if r.size else np.zeros(0, np.int64)
    out = np.zeros((x.shape[0], nrow))
    if r.size:
        out[:, r[starts]] = np.add.reduceat(contrib, starts, axis=1)
    return out


def _termination_holds(b, x, y):
    P, A = b["P"], b["A"]
    n, m = b["n"], b["m"]
    pr, pc = _csc_rows_cols(P)
    ar, ac = _csc_rows_cols(A)
    Px = _matvec(pr, pc, b["Px"], x, n)
    off = pr != pc  # full symmetric P from its upper triangle
    Px += _matvec(pc[off], pr[off], b["Px"][:, off], x, n)
    Ax = _matvec(ar, ac, b["Ax"], x, m)
    Aty = _matvec(ac, ar, b["Ax"], y, n)
    q = b["q"]
    inf = lambda v: np.abs(v).max(axis=1)  # noqa: E731
    r_dua = inf(Px + q + Aty)
    tol_dua = EPS + EPS * np.maximum(np.maximum(inf(Px), inf(Aty)), inf(q))
    lo = np.maximum(b["l"], -1e30)
    up = np.minimum(b["u"], 1e30)
    dist = inf(np.maximum(lo - Ax, 0.0) + np.maximum(Ax - up, 0.0))
    tol_pri = (EPS + EPS * inf(Ax)) / (1.0 - EPS)
    return r_dua <= tol_dua * (1 + 1e-9) + SLACK, dist <= tol_pri * (1 + 1e-9) + SLACK, r_dua / tol_dua, dist / tol_pri


def termination_holds(b, x, y):
    """(dual ok, primal ok) per instance; shared with the CPU test of this checker."""
    ok_d, ok_p, _, _ = _termination_holds(b, x, y)
    return ok_d, ok_p


def test_cfg3_full_batch_meets_the_termination_test():
    b = mpc.make_batch(3)  # configs[2]: B = 65536
    B = b["Px"].shape[0]
    assert B == 65536
    s = {k: v for k, v in b["settings"].items() if k != "verbose"}
    h = OSQPBatch()
    h.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
    r1 = h.solve()
    assert (r1.status_val == 1).all()
    ok_d, ok_p, fd, fp = _termination_holds(b, r1.x, r1.y)
    assert ok_d.all(), (np.flatnonzero(~ok_d)[:10], fd.max())
    assert ok_p.all(), (np.flatnonzero(~ok_p)[:10], fp.max())
    # a receding-horizon step: initial states moved, bounds updated, solved again (warm,
    # dispatched longest-previous-first from the first solve's iteration counts)
    rng = np.random.default_rng(11)
    l, u = b["l"].copy(), b["u"].copy()
    x0 = -l[:, :5] + rng.uniform(-0.02, 0.02, (B, 5))
    l[:, :5] = -x0
    u[:, :5] = -x0
    h.update(l=l, u=u)
    r2 = h.solve()
    assert (r2.status_val == 1).all()
    b2 = dict(b, l=l, u=u)
    ok_d, ok_p, fd, fp = _termination_holds(b2, r2.x, r2.y)
    assert ok_d.all(), (np.flatnonzero(~ok_d)[:10], fd.max())
    assert ok_p.all(), (np.flatnonzero(~ok_p)[:10], fp.max())
    # the oracle on a sample of the first solve
    idx = np.random.default_rng(1).choice(B, 256, replace=False)
    bo = pyoracle.solve_batch(b["P"], b["A"], b["Px"][idx], b["q"][idx], b["Ax"][idx], b["l"][idx], b["u"][idx],
                              nthreads=16, **s)
    assert np.mean(bo.iter == r1.iter[idx]) >= 0.99
    same = bo.iter == r1.iter[idx]
    du = np.abs(r1.x[idx][:, b["u_block"]] - bo.x[:, b["u_block"]]).max(axis=1)
    assert np.all(du[same] < 1e-4), du.max()


def _stage_shift(v, N, nxa, nu, groups):
    """One-stage shift of incremental-layout iterates (mpcqp_incr_warm_shift_device; the
    reference's horizon shift, mpc_dynamics.py:589-610)."""
    B = v.shape[0]
    out = []
    for g in range(groups):
        blk = v[:, g * (N + 1) * nxa:(g + 1) * (N + 1) * nxa].reshape(B, N + 1, nxa)
        out.append(np.concatenate([blk[:, 1:], blk[:, -1:]], 1).reshape(B, -1))
    du = v[:, groups * (N + 1) * nxa:].reshape(B, N, nu)
    out.append(np.concatenate([du[:, 1:], du[:, -1:]], 1).reshape(B, -1))
    return np.concatenate(out, 1)


def test_cfg5_full_batch_warm_meets_the_termination_test():
    """configs[4] at full size (B = 8192 incremental dynamic QPs, N = 50), as bench.py times
    it: a cold solve, then the solution shifted one stage (the warm start of SURVEY.md §8d
    D2) and the next step's QP -- initial states jittered +-2 % of the D2 ranges, as
    bench.py::bound_sequence -- solved from it, dispatched longest-previous-first from the
    cold solve's iteration counts.  Every instance of both solves: status solved (the oracle
    solves a 512-instance sample of this batch cold and warm with no other status) and OSQP's
    termination test recomputed on the host.  An oracle sample of 128 pins the warm solve's
    iteration counts and du."""
    import bench
    b = mpc.make_batch(5)
    B, N = b["Px"].shape[0], b["N"]
    assert B == 8192
    s = {k: v for k, v in b["settings"].items() if k != "verbose"}
    h = OSQPBatch()
    h.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
    r1 = h.solve()
    assert (r1.status_val == 1).all(), np.unique(r1.status_val, return_counts=True)
    ok_d, ok_p, fd, fp = _termination_holds(b, r1.x, r1.y)
    assert ok_d.all(), (np.flatnonzero(~ok_d)[:10], fd.max())
    assert ok_p.all(), (np.flatnonzero(~ok_p)[:10], fp.max())
    xs, ys = _stage_shift(r1.x, N, 8, 2, 1), _stage_shift(r1.y, N, 8, 2, 2)
    x0 = bench.x0_sequence(b, 2, bench.instance_seed(5, 0))[1]
    l, u = b["l"].copy(), b["u"].copy()
    l[:, :x0.shape[1]] = -x0
    u[:, :x0.shape[1]] = -x0
    h.update(l=l, u=u)
    h.warm_start(x=xs, y=ys)
    r2 = h.solve()
    assert (r2.status_val == 1).all(), np.unique(r2.status_val, return_counts=True)
    assert r2.iter.mean() < r1.iter.mean()
    b2 = dict(b, l=l, u=u)
    ok_d, ok_p, fd, fp = _termination_holds(b2, r2.x, r2.y)
    assert ok_d.all(), (np.flatnonzero(~ok_d)[:10], fd.max())
    assert ok_p.all(), (np.flatnonzero(~ok_p)[:10], fp.max())
    idx = np.random.default_rng(2).choice(B, 128, replace=False)
    bo = pyoracle.solve_batch(b["P"], b["A"], b["Px"][idx], b["q"][idx], b["Ax"][idx], l[idx], u[idx],
                              nthreads=16, x0=xs[idx], y0=ys[idx], **s)
    same = bo.iter == r2.iter[idx]
    assert (bo.status_val == 1).all() and same.mean() >= 0.97, (bo.iter[~same], r2.iter[idx][~same])
    du = np.abs(r2.x[idx][:, b["u_block"]] - bo.x[:, b["u_block"]]).max(axis=1)
    assert np.all(du[same] < 1e-4), du.max()
