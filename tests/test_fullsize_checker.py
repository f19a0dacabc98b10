"""CPU check of the termination-test checker (tests/parity.py, used by the GPU parity tests): the oracle's own
"solved" results (OSQP 0.6 restatement) satisfy it on a small slack batch, and a perturbed
solution fails it."""
import numpy as np

import pyoracle
from osqp_amd import mpc
from parity import termination_holds


def test_checker_accepts_oracle_solutions_and_rejects_perturbed_ones():
    b = mpc.make_batch(3, B=48, seed=4)
    s = {k: v for k, v in b["settings"].items() if k != "verbose"}
    r = pyoracle.solve_batch(b["P"], b["A"], b["Px"], b["q"], b["Ax"], b["l"], b["u"], nthreads=4, **s)
    assert (r.status_val == 1).all()
    ok_d, ok_p = termination_holds(b, r.x, r.y)
    assert ok_d.all() and ok_p.all()
    y = r.y.copy()
    y[:, 7] += 1.0
    ok_d, _ = termination_holds(b, r.x, y)
    assert not ok_d.any()
    x = r.x.copy()
    x[:, 0] += 1.0  # the initial-state row: an equality
    _, ok_p = termination_holds(b, x, r.y)
    assert not ok_p.any()
