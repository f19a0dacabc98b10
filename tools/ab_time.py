#!/usr/bin/env python3
"""Kernel-time A/B harness (GPU only, diagnostic): the same batch solved `reps` times
with identity dispatch, setup and solve as separate calls; prints the mean HIP-event
time of the setup and solve launches.  The package is taken from --pkg (default: this
repository's), so two builds can be timed in one process run each on the same box.

  python tools/ab_time.py --config 3 --batch 16384 [--pkg /path/to/python-mpc_amd]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--pkg", default=os.path.join(ROOT, "python-mpc_amd"))
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    sys.path.insert(0, a.pkg)
    os.environ["MPCQP_DISPATCH"] = "identity"
    import numpy as np
    import torch
    import osqp_amd
    from osqp_amd import DeviceBatch, mpc, _drop_common_zeros
    spec = mpc.CONFIGS[a.config]
    B = a.batch or spec["B"]
    b = mpc.make_batch(a.config, B=B, seed=1000 * a.config)
    P, Px = _drop_common_zeros(b["P"], b["Px"])
    A, Ax = _drop_common_zeros(b["A"], b["Ax"])
    s = {k: v for k, v in b["settings"].items() if k != "verbose"}
    dev = torch.device("cuda", 0)
    X = [torch.from_numpy(np.ascontiguousarray(v)).to(dev) for v in (Px, Ax, b["q"], b["l"], b["u"])]
    o = (torch.empty((B, b["n"]), dtype=torch.float64, device=dev), torch.empty((B, b["m"]), dtype=torch.float64, device=dev),
         torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.int32, device=dev))
    h = DeviceBatch(P, A, B, device=0, **s)
    h.setup(*X)
    h.solve(*o)
    h.synchronize()
    h.timing(True)
    for _ in range(a.reps):
        h.setup(*X)
        h.solve(*o)
    h.synchronize()
    t = h.timing_read()
    print(f"{a.tag} {os.path.basename(os.path.dirname(osqp_amd.__file__))} config {a.config} B={B}: "
          f"setup {t['setup_ms'] / t['n_setup']:.3f} ms solve {t['solve_ms'] / t['n_solve']:.3f} ms "
          f"iters mean {o[3].float().mean().item():.1f}", flush=True)


if __name__ == "__main__":
    main()
