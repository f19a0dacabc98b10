"""Solves of tests/test_skew.py, run once with the production library and once (in a child
process, MPCQP_BUILD=skew or prof) with a diagnostic build -- TEST INFRASTRUCTURE ONLY.
Every kernel family with hand-offs between waves: the four-wave kernel (cfg 2, and the
slack layout's reduced system), the two-wave and eight-wave kernels, the 256-thread
register-sweep kernel, the 512-thread long-horizon kernel."""
import os
import sys

import numpy as np

CASES = [  # (name, config, batch, MPCQP_VARIANT or None, MPCQP_ELIM)
    ("w4_cfg2", 2, 512, None, None),
    ("w4_slack_elim", 3, 256, None, None),
    ("w2_cfg2", 2, 256, "10", None),
    ("w8_slack", 3, 128, "18", "0"),
    ("sweep256_slack", 3, 128, "2", "0"),
    ("big_cfg5", 5, 32, "12", None),
]


def run(name, cfg, B, variant, elim):
    from osqp_amd import OSQPBatch, mpc
    for k, v in (("MPCQP_VARIANT", variant), ("MPCQP_ELIM", elim)):
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    b = mpc.make_batch(cfg, B=B, seed=71)
    s = {k: v for k, v in b["settings"].items() if k != "verbose"}
    h = OSQPBatch()
    h.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
    r1 = h.solve()
    l, u = b["l"].copy(), b["u"].copy()
    l[:, :2] *= 0.95
    u[:, :2] *= 0.95
    h.update(l=l, u=u)
    r2 = h.solve()  # warm-started, in the dispatch order the first solve left
    res = {f"{name}_{k}{i}": getattr(r, k) for i, r in enumerate((r1, r2)) for k in ("x", "y", "iter", "status_val")}
    if os.environ.get("MPCQP_PHASE_PROF") == "1":
        res[f"{name}_phase_times"] = h.phase_times()
    return res


def main(out):
    res = {}
    for c in CASES:
        res.update(run(*c))
    np.savez(out, **res)


if __name__ == "__main__":
    HERE = os.path.dirname(os.path.abspath(__file__))
    ROOT = os.path.dirname(HERE)
    sys.path[:0] = [os.path.join(ROOT, "python-mpc_amd"), HERE]
    main(sys.argv[1])
