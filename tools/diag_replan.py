#!/usr/bin/env python3
"""Diagnostic (GPU): update_settings(polish=True) on an eliminated-slack handle (api.hip::
replan_plain) against the same call sequences without the re-plan, each beside the oracle.

  python tools/diag_replan.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("python-mpc_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np  # noqa: E402
import pyoracle  # noqa: E402
from conftest import load_golden  # noqa: E402
from osqp_amd import OSQP  # noqa: E402

g = load_golden("slack_n20.npz")
P, A, q, l, u = g["P"], g["A"], g["q"], g["l"], g["u"]
q2, l2, u2 = g["upd_q"][1], g["upd_l"][1], g["upd_u"][1]


def run(seq, elim="1"):
    os.environ["MPCQP_ELIM"] = elim
    d, o = OSQP(), pyoracle.OSQP()
    for obj in (d, o):
        kw = dict(warm_start=True)
        if "P0" in seq:
            kw["polish"] = True
        obj.setup(P, q, A, l, u, **kw)
    out = []
    for op in seq:
        if op == "P0":
            continue
        for obj in (d, o):
            if op == "S":
                pass
            elif op == "P":
                obj.update_settings(polish=True)
            elif op == "U":
                obj.update(q=q2, l=l2, u=u2)
        if op == "S":
            rd, ro = d.solve(), o.solve()
            out.append(f"dev {rd.info.status}/{rd.info.iter} orc {ro.info.status}/{ro.info.iter} "
                       f"|dx| {np.max(np.abs(rd.x - ro.x)):.2e} |dy| {np.max(np.abs(rd.y - ro.y)):.2e}")
    if hasattr(d, "plan_info"):
        try:
            out.append(str(d.plan_info()))
        except Exception as e:  # noqa: BLE001
            out.append(repr(e))
    return out


for name, seq, elim in [("polish at setup, S U S", ["P0", "S", "U", "S"], "1"),
                        ("no polish, S U S", ["S", "U", "S"], "1"),
                        ("replan, S P S", ["S", "P", "S"], "1"),
                        ("replan, S P U S", ["S", "P", "U", "S"], "1"),
                        ("replan before any solve, P S", ["P", "S"], "1"),
                        ("plain plan, S P U S", ["S", "P", "U", "S"], "0")]:
    print(name)
    for line in run(seq, elim):
        print("   ", line)
