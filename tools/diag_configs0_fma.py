#!/usr/bin/env python3
"""configs[0] loop (tests/test_gpu_parity.py::_slack_script_loop, 1500 steps at N = 20):
how far the oracle moves under a rounding-level change of its own arithmetic.  The oracle
(oracle/osqp_oracle.c, built -march=x86-64-v2: no FMA) is rebuilt into a temporary
directory with -march=x86-64-v3 -ffp-contract=fast (FMA contraction) and both run the
loop; the FMA build once on its own plant states and once driven along the standard
build's, as the GPU test drives the device.  CPU only; diagnostic (no test imports it)."""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys
sys.path[:0] = [sys.argv[1] + "/tests", sys.argv[1] + "/python-mpc_amd", sys.argv[1] + "/oracle"]
import numpy as np, pyoracle
if sys.argv[2] != "-": pyoracle._LIB = sys.argv[2]
from test_gpu_parity import _slack_script_loop
states = np.load(sys.argv[4]) if sys.argv[4] != "-" else None
o, xo = _slack_script_loop(pyoracle, states=states)
np.save(sys.argv[3] + "_out.npy", o); np.save(sys.argv[3] + "_xs.npy", xo)
'''


def main():
    import numpy as np
    with tempfile.TemporaryDirectory() as td:
        lib = os.path.join(td, "liboracle_fma.so")
        subprocess.check_call(["gcc", "-O3", "-march=x86-64-v3", "-ffp-contract=fast", "-fPIC", "-shared", "-o", lib,
                               os.path.join(ROOT, "oracle", "osqp_oracle.c"), "-lm", "-lpthread"])
        child = os.path.join(td, "child.py")
        open(child, "w").write(CHILD)
        run = lambda tag, L, st: subprocess.check_call([sys.executable, child, ROOT, L, os.path.join(td, tag), st])
        run("std", "-", "-")
        run("fma", lib, "-")
        run("fma_on_std", lib, os.path.join(td, "std_xs.npy"))
        o = np.load(os.path.join(td, "std_out.npy"))
        for tag in ("fma", "fma_on_std"):
            g = np.load(os.path.join(td, tag + "_out.npy"))
            it = np.flatnonzero(g[:, 1] != o[:, 1])
            d = np.abs(g[:, 0] - o[:, 0])
            print(f"{tag}: iteration mismatches {it.size} {it[:10].tolist()}, du_0 diff max {d.max():.3e} at step "
                  f"{int(d.argmax())}, steps > 1e-4: {int((d > 1e-4).sum())}")


if __name__ == "__main__":
    main()
