#!/usr/bin/env python3
"""Per-call latency legs of bench.py (bench.latency_leg: a fresh OSQP() + setup() + solve() of
ONE QP per call, cfg 2 and cfg 5) as one JSON line, for same-box A/Bs of the host call path."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "python-mpc_amd"), os.path.join(ROOT, "oracle"), ROOT]

if __name__ == "__main__":
    import bench
    out = {"env": {k: v for k, v in os.environ.items() if k.startswith("MPCQP_")}}
    for cfg in [int(c) for c in (sys.argv[1:] or ["2", "5"])]:
        r = bench.latency_leg(cfg, reps=30)
        out[f"cfg{cfg}"] = {k: r["gpu"][k] for k in ("call_ms", "setup_ms", "solve_ms", "iters", "solve_us_per_iter")}
        out[f"cfg{cfg}"]["cpu_call_ms"] = r["cpu"]["call_ms"]
        out[f"cfg{cfg}"]["cpu_solve_us_per_iter"] = r["cpu"]["solve_us_per_iter"]
    print(json.dumps(out))
