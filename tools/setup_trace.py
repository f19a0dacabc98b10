#!/usr/bin/env python3
"""Diagnostic (GPU): the host-side stages of mpcqp_setup_batch (MPCQP_SETUP_TRACE=1, api.hip
SetupTrace) for one QP of the given config, a few setups in a row (the later ones hit the
plan cache and the resource pool).

  python tools/setup_trace.py [config]
"""
import os
import sys

os.environ["MPCQP_SETUP_TRACE"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-mpc_amd"))
from osqp_amd import OSQP, mpc  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 5
b = mpc.make_batch(cfg, B=1, seed=1)
P, A = b["P"].copy(), b["A"].copy()
P.data, A.data = b["Px"][0].copy(), b["Ax"][0].copy()
q, l, u = b["q"][0].copy(), b["l"][0].copy(), b["u"][0].copy()
for k in range(4):
    print(f"--- setup {k}", file=sys.stderr, flush=True)
    o = OSQP()
    o.setup(P, q, A, l, u, warm_start=True, verbose=False)
    o.solve()
    del o
