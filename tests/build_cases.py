"""Solves run under one of the library's builds in a child process -- TEST INFRASTRUCTURE
ONLY.  The production library (libmpcqp.so) is what the parent test process loads; the
other builds (python-mpc_amd/csrc/Makefile) are selected by MPCQP_BUILD at import, so
they run here, in a child:

  exp   the production kernels plus the variants measured and not taken (one-wave 8/9,
        two-sided two-wave 14, dense inverse 16, eight-wave 18)
  skew  barrier-race build (every workgroup barrier skews the waves), experimental too
  prof  phase-timer build, experimental too

CASES are the production kernel families with hand-offs between waves (tests/test_skew.py
compares them bit for bit between builds): the four-wave kernel (cfg 2, and the slack
layout's reduced system), the two-wave kernel, the 256-thread register-sweep kernel, the
512-thread long-horizon kernel.  EXP_CASES: the eight-wave kernel (variant 18)."""
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

CASES = [  # (name, config, batch, MPCQP_VARIANT or None, MPCQP_ELIM)
    ("w4_cfg2", 2, 512, None, None),
    ("w4_slack_elim", 3, 256, None, None),
    ("w2_cfg2", 2, 256, "10", None),
    ("sweep256_slack", 3, 128, "2", "0"),
    ("big_cfg5", 5, 32, "12", None),
]
EXP_CASES = [
    ("w8_slack", 3, 128, "18", "0"),
]


def _env(variant, elim):
    for k, v in (("MPCQP_VARIANT", variant), ("MPCQP_ELIM", elim)):
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


def run(name, cfg, B, variant, elim):
    """A cold solve and a warm re-solve (dispatched in the order the first one left)."""
    from osqp_amd import OSQPBatch, mpc
    _env(variant, elim)
    b = mpc.make_batch(cfg, B=B, seed=71)
    s = {k: v for k, v in b["settings"].items() if k != "verbose"}
    h = OSQPBatch()
    h.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
    r1 = h.solve()
    l, u = b["l"].copy(), b["u"].copy()
    l[:, :2] *= 0.95
    u[:, :2] *= 0.95
    h.update(l=l, u=u)
    r2 = h.solve()
    res = {f"{name}_{k}{i}": getattr(r, k) for i, r in enumerate((r1, r2)) for k in ("x", "y", "iter", "status_val")}
    if os.environ.get("MPCQP_PHASE_PROF") == "1":
        res[f"{name}_phase_times"] = h.phase_times()
    return res


def run_batch(name, cfg, B, variant, settings):
    """One solve of mpc.make_batch(cfg, B) (default seed) with the variant forced."""
    from osqp_amd import OSQPBatch, mpc
    _env(variant, None)
    b = mpc.make_batch(cfg, B=B)
    h = OSQPBatch()
    h.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **settings)
    r = h.solve()
    info = h.plan_info()
    return {f"{name}_x": r.x, f"{name}_y": r.y, f"{name}_iter": r.iter, f"{name}_status_val": r.status_val,
            f"{name}_variant": np.int32(info["variant"])}


def in_build(build, specs, out, timeout=240, extra_env=None):
    """Run specs -- ("case", *CASES entry) or ("batch", name, cfg, B, variant, settings) --
    in a child process under MPCQP_BUILD=build (plus extra_env: switches the library reads
    once per process, such as MPCQP_DENSE_W4); returns the saved arrays."""
    env = dict(os.environ, MPCQP_BUILD=build)
    for k in ("MPCQP_VARIANT", "MPCQP_ELIM", "MPCQP_PHASE_PROF", "MPCQP_DENSE_W4"):
        env.pop(k, None)
    env.update(extra_env or {})
    if build == "prof":
        env["MPCQP_PHASE_PROF"] = "1"
    subprocess.run([sys.executable, os.path.join(HERE, "build_cases.py"), str(out), json.dumps(specs)], env=env,
                   check=True, timeout=timeout)
    with np.load(out) as z:
        return {k: z[k] for k in z.files}


def main(out, specs):
    res = {}
    for kind, *args in specs:
        res.update(run(*args) if kind == "case" else run_batch(*args))
    np.savez(out, **res)


if __name__ == "__main__":
    ROOT = os.path.dirname(HERE)
    sys.path[:0] = [os.path.join(ROOT, "python-mpc_amd"), HERE]
    main(sys.argv[1], json.loads(sys.argv[2]))
