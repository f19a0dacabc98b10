"""Barrier races made deterministic to catch.

The skew build (python-mpc_amd/csrc/device_common.h, MPCQP_SKEW; make skew ->
libmpcqp_skew.so) sleeps about half of a workgroup's waves, a different half at every
barrier, for ~1,300 cycles after each workgroup barrier.  A hand-off between waves that
is not ordered by a barrier then goes wrong within a few barriers -- the round-2 y-park
race showed up in ~1 of 4 runs of the production build -- while every ordered hand-off
gives the same bits.  So: each kernel family's results with the skew build (a child
process, MPCQP_BUILD=skew) must equal the production build's bit for bit, over a cold
solve and a warm re-solve dispatched in the order the first one left.

The same harness runs the phase-timer build (MPCQP_BUILD=prof, MPCQP_PHASE_PROF=1; make
prof -> libmpcqp_prof.so) over the same six kernel families: its only extra global
accesses are the per-instance timer slots (p.prof[b * kProfSlots + k], B x 16 int64 in
the workspace), so it too must reproduce the production bits, and every instance's
timers must be filled (the round-2 memory aperture violation came
from the phase-timer build of a gather-length-5 instantiation that no longer exists;
solve_wave.hip::lists_fit now refuses a launch whose compile-time list lengths are
shorter than the plan's).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("build", ["skew", "prof"])
def test_diagnostic_build_is_bit_identical(tmp_path, build):
    import osqp_amd
    dlib = os.path.join(os.path.dirname(osqp_amd.LIB_PATH), f"libmpcqp_{build}.so")
    assert os.path.exists(dlib), f"build it: make -C python-mpc_amd/csrc {build}"
    out = tmp_path / f"{build}.npz"
    env = dict(os.environ, MPCQP_BUILD=build)
    for k in ("MPCQP_VARIANT", "MPCQP_ELIM", "MPCQP_PHASE_PROF"):
        env.pop(k, None)
    if build == "prof":
        env["MPCQP_PHASE_PROF"] = "1"
    subprocess.run([sys.executable, os.path.join(HERE, "skew_cases.py"), str(out)], env=env, check=True, timeout=240)
    import skew_cases
    saved = {k: os.environ.get(k) for k in ("MPCQP_VARIANT", "MPCQP_ELIM")}
    try:
        ref = {}
        for c in skew_cases.CASES:
            ref.update(skew_cases.run(*c))
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    got = np.load(out)
    bad = [k for k in ref if not np.array_equal(ref[k], got[k], equal_nan=True)]
    assert not bad, bad
    if build == "prof":
        for c in skew_cases.CASES:
            t = got[f"{c[0]}_phase_times"]
            assert np.all(t[:, 6] > 0) and np.all(t[:, 7] > 0), c[0]  # total cycles, wall ticks
