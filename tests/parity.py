"""Shared parity checks of the device solver against the oracle (not a test module).

SURVEY.md §8c C4 (ii): agreement in status and iteration count is the strong check, but an
instance on which the two disagree must not pass silently.  `check_agreement` therefore

* records the observed agreement fractions (printed in pytest's terminal summary by
  conftest.py, so every GPU log carries them);
* requires the fractions to reach `min_match`;
* where both agree: the north-star bound ||u - u_ref||_inf < 1e-4;
* where they DISAGREE (status or iteration count): the device must report "solved" (or the
  oracle's own status), its returned (x, y) must pass OSQP 0.6's termination test for
  "solved" recomputed on the host from the instance's CSC values (`termination_holds`), and,
  given `tight` (the oracle's solution of the same instances at eps 1e-9: the optimum u*),
  the device's controls must be as close to u* as the oracle's own, up to a factor:
  ||u - u*||_inf <= 10 ||u_ref - u*||_inf + 1e-4.
  (Not ||u - u_ref|| <= eps_abs + eps_rel ||u_ref||: OSQP's stopping rule bounds residuals,
  not the distance between two points that both pass it.  On cfg 5 warm -- two instances of a
  128-sample whose counts part by one check interval -- the device and oracle controls
  differ by 0.03 while both pass the termination test; the measured distances to u* are
  printed with the agreement fractions.)

`termination_holds` (OSQP 0.6 check_termination, unscaled residuals):

  dual:   ||P x + q + A'y||_inf <= eps_abs + eps_rel * max(||P x||, ||A'y||, ||q||)
  primal: dist(A x, [l, u])_inf <= ||A x - z||_inf <= eps_abs + eps_rel * max(||A x||, ||z||),
          and with ||z|| <= ||A x|| + ||A x - z||:  dist <= (eps_abs + eps_rel ||A x||) / (1 - eps_rel)
"""
import numpy as np

U_TOL = 1e-4
EPS = 1e-3
SLACK = 1e-9  # host recomputation of the residuals (fp64 sums in another order)

RECORDS = []  # (label, n, status agreement, iteration agreement, mismatches, max du where equal, note)


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


def termination_detail(b, x, y, eps=EPS):
    """(dual ok, primal ok, dual residual / tolerance, primal distance / tolerance) per instance."""
    P, A = b["P"], b["A"]
    n, m = b["n"], b["m"]
    Pv = np.broadcast_to(b["Px"], (x.shape[0], P.nnz))
    Av = np.broadcast_to(b["Ax"], (x.shape[0], A.nnz))
    pr, pc = _csc_rows_cols(P)
    ar, ac = _csc_rows_cols(A)
    Px = _matvec(pr, pc, Pv, x, n)
    off = pr != pc  # full symmetric P from its upper triangle
    Px += _matvec(pc[off], pr[off], Pv[:, off], x, n)
    Ax = _matvec(ar, ac, Av, x, m)
    Aty = _matvec(ac, ar, Av, y, n)
    q = b["q"]
    inf = lambda v: np.abs(v).max(axis=1)  # noqa: E731
    r_dua = inf(Px + q + Aty)
    tol_dua = eps + eps * np.maximum(np.maximum(inf(Px), inf(Aty)), inf(q))
    lo = np.maximum(b["l"], -1e30)
    up = np.minimum(b["u"], 1e30)
    dist = inf(np.maximum(lo - Ax, 0.0) + np.maximum(Ax - up, 0.0))
    tol_pri = (eps + eps * inf(Ax)) / (1.0 - eps)
    return (r_dua <= tol_dua * (1 + 1e-9) + SLACK, dist <= tol_pri * (1 + 1e-9) + SLACK, r_dua / tol_dua,
            dist / tol_pri)


def termination_holds(b, x, y):
    """(dual ok, primal ok) per instance."""
    ok_d, ok_p, _, _ = termination_detail(b, x, y)
    return ok_d, ok_p


def subset(b, idx):
    """The instances idx of batch dict b (per-instance value arrays sliced)."""
    out = dict(b)
    for k in ("Px", "Ax", "q", "l", "u"):
        v = np.asarray(b[k])
        out[k] = v[idx] if v.ndim == 2 else v
    return out


def check_agreement(label, b, x, y, status, iters, bo, min_match=1.0, eps=EPS, tight=None):
    """Device results (x, y, status, iters over the instances of b) against the oracle's `bo`
    (pyoracle.solve_batch over the same instances); see the module docstring.  `tight(idx)`:
    the oracle's x at eps 1e-9 for instances idx (the disagreeing ones).  Returns du."""
    ub = b["u_block"]
    same_status = status == bo.status_val
    same_iter = iters == bo.iter
    ok = np.isfinite(bo.x).all(axis=1)
    du = np.abs(x[:, ub] - bo.x[:, ub]).max(axis=1)
    agree = same_status & same_iter
    diff = np.flatnonzero(~agree)
    rec = [label, int(status.size), float(same_status.mean()), float(same_iter.mean()), int(diff.size),
           float(du[ok & agree].max()) if (ok & agree).any() else 0.0, ""]
    RECORDS.append(rec)
    assert same_status.mean() >= min_match, (label, status[~same_status][:8], bo.status_val[~same_status][:8])
    assert same_iter.mean() >= min_match, (label, iters[~same_iter][:8], bo.iter[~same_iter][:8])
    assert np.all(du[ok & agree] < U_TOL), (label, du[ok & agree].max())
    if diff.size:
        st = status[diff]
        assert np.all((st == 1) | (st == bo.status_val[diff])), (label, diff, st, bo.status_val[diff])
        solved = np.flatnonzero(st == 1)
        if solved.size:
            assert y is not None, (label, "disagreeing instances and no y to check them with")
            d = diff[solved]
            ok_d, ok_p, fd, fp = termination_detail(subset(b, d), x[d], y[d], eps)
            assert ok_d.all() and ok_p.all(), (label, d, fd, fp)
        if tight is not None:
            xs = np.asarray(tight(diff))
            dd = np.abs(x[diff][:, ub] - xs[:, ub]).max(axis=1)
            do = np.abs(bo.x[diff][:, ub] - xs[:, ub]).max(axis=1)
            rec[6] = "; |u - u*| device " + ", ".join(f"{v:.1e}" for v in dd) + " / oracle " + \
                     ", ".join(f"{v:.1e}" for v in do)
            assert np.all(dd <= 10 * do + U_TOL), (label, diff, dd, do)
    return du
