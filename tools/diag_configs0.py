#!/usr/bin/env python3
"""configs[0] loop (tests/test_gpu_parity.py::_slack_script_loop, 1500 steps at N = 20):
where the device's du_0 departs from the oracle's, with the loop driven along the oracle's
plant states, for the eliminated-slack plan and the full plan (MPCQP_ELIM=0); and the
oracle against itself under 1e-14 relative state perturbations (the loop's own
sensitivity).  Diagnostic, GPU only; prints one summary per mode."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "tests"), os.path.join(ROOT, "python-mpc_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import pyoracle  # noqa: E402
from test_gpu_parity import _slack_script_loop  # noqa: E402


def shim():
    spec = importlib.util.spec_from_file_location("osqp", os.path.join(ROOT, "python-mpc_amd", "shim", "osqp.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def report(tag, o, g, xo):
    d = np.abs(g[:, 0] - o[:, 0])
    it = np.flatnonzero(g[:, 1] != o[:, 1])
    big = np.flatnonzero(d > 1e-4)
    xn = np.abs(xo[:-1]).max(axis=1)
    print(f"{tag}: iter mismatches {len(it)} (first {it[:5].tolist()}), du diff max {d.max():.3e} at step "
          f"{d.argmax()}, steps > 1e-4: {len(big)}, > 1e-6: {(d > 1e-6).sum()}; |x0|_inf at the worst step "
          f"{xn[d.argmax()]:.1f}; tolerance eps_abs + eps_rel |x0|_inf there {1e-3 + 1e-3 * xn[d.argmax()]:.3e}; "
          f"max du diff / that tolerance {np.max(d / (1e-3 + 1e-3 * xn)):.3f}", flush=True)
    for s in big[:12]:
        print(f"   step {s}: du {o[s, 0]:+.6e} vs {g[s, 0]:+.6e}  iters {int(o[s, 1])}/{int(g[s, 1])}  |x0| {xn[s]:.1f}")


def main():
    o, xo = _slack_script_loop(pyoracle)
    rng = np.random.default_rng(1)
    p, _ = _slack_script_loop(pyoracle, states=xo * (1 + 1e-14 * rng.standard_normal(xo.shape)))
    report("oracle vs oracle (states x (1 + 1e-14 N(0,1)))", o, p, xo)
    for elim in ("1", "0"):
        os.environ["MPCQP_ELIM"] = elim
        g, _ = _slack_script_loop(shim(), states=xo)
        report(f"device (MPCQP_ELIM={elim}) vs oracle", o, g, xo)


if __name__ == "__main__":
    main()
