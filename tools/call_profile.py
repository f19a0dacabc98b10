"""Diagnostic: where one cfg-5 (or cfg-2) QP call's host time goes -- a fresh osqp_amd.OSQP() +
setup() + solve() per call as bench.py's latency leg makes it, under cProfile, plus the
median of each phase.  python3 tools/call_profile.py [cfg] [reps]"""
import cProfile
import os
import pstats
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-mpc_amd"))
from osqp_amd import OSQP, mpc  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 5
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
b = mpc.make_batch(cfg, B=1, seed=1)
P, A = b["P"].copy(), b["A"].copy()
P.data, A.data = b["Px"][0].copy(), b["Ax"][0].copy()
q, l, u = b["q"][0].copy(), b["l"][0].copy(), b["u"][0].copy()
settings = {k: v for k, v in b["settings"].items() if k != "verbose"}


def call():
    t0 = time.perf_counter()
    o = OSQP()
    t1 = time.perf_counter()
    o.setup(P, q, A, l, u, **settings)
    t2 = time.perf_counter()
    r = o.solve()
    t3 = time.perf_counter()
    del o
    return t1 - t0, t2 - t1, t3 - t2, r.info.iter


for _ in range(5):
    call()
ts = np.array([call()[:3] for _ in range(reps)])
print("median ms: OSQP() %.3f setup %.3f solve %.3f total %.3f"
      % tuple(1e3 * np.array(np.median(ts, 0).tolist() + [np.median(ts.sum(1))])))
pr = cProfile.Profile()
pr.enable()
for _ in range(reps):
    call()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
