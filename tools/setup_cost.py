#!/usr/bin/env python3
"""Setup-kernel time vs the number of Ruiz passes (GPU only, diagnostic).

  python tools/setup_cost.py --config 2 [--batch B]

Times mpcqp_setup_device (HIP events on the handle's stream) at scaling = 0, 1, 2, 5,
10: the slope is the cost of one Ruiz pass over the batch, the intercept the loads,
bounds classification and stores.  MPCQP_SETUP_STAGED=1 selects the staged-index kernel.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-mpc_amd"))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    from osqp_amd import DeviceBatch, mpc, _drop_common_zeros
    spec = mpc.CONFIGS[a.config]
    B = a.batch or spec["B"]
    b = mpc.make_batch(a.config, B=B, seed=5)
    P, Px = _drop_common_zeros(b["P"], b["Px"])
    A, Ax = _drop_common_zeros(b["A"], b["Ax"])
    s = {k: v for k, v in b["settings"].items() if k != "verbose"}
    dev = torch.device("cuda", 0)
    X = [torch.from_numpy(np.ascontiguousarray(v)).to(dev) for v in (Px, Ax, b["q"], b["l"], b["u"])]
    for sc in (0, 1, 2, 5, 10):
        h = DeviceBatch(P, A, B, device=0, **dict(s, scaling=sc))
        h.setup(*X)
        h.synchronize()
        h.timing(True)
        for _ in range(a.reps):
            h.setup(*X)
        h.synchronize()
        t = h.timing_read()
        h.timing(False)
        print(f"config {a.config} B={B} scaling={sc}: setup {t['setup_ms'] / t['n_setup'] * 1e3:.1f} us",
              flush=True)


if __name__ == "__main__":
    main()
