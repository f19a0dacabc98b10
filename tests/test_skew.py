"""Barrier races made deterministic to catch.

The skew build (python-mpc_amd/csrc/device_common.h, MPCQP_SKEW; make skew ->
libmpcqp_skew.so) sleeps about half of a workgroup's waves, a different half at every
barrier, for ~1,300 cycles after each workgroup barrier.  A hand-off between waves that
is not ordered by a barrier then goes wrong within a few barriers -- the round-2 y-park
race showed up in ~1 of 4 runs of the production build -- while every ordered hand-off
gives the same bits.  So: each kernel family's results with the skew build (a child
process, MPCQP_BUILD=skew) must equal the production build's bit for bit, over a cold
solve and a warm re-solve dispatched in the order the first one left.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_skew_build_is_bit_identical(tmp_path):
    import osqp_amd
    skew_lib = os.path.join(os.path.dirname(osqp_amd.LIB_PATH), "libmpcqp_skew.so")
    assert os.path.exists(skew_lib), "build it: make -C python-mpc_amd/csrc skew"
    out = tmp_path / "skew.npz"
    env = dict(os.environ, MPCQP_BUILD="skew")
    for k in ("MPCQP_VARIANT", "MPCQP_ELIM", "MPCQP_PHASE_PROF"):
        env.pop(k, None)
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
