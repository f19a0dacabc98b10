#!/usr/bin/env python3
"""Diagnostic: is cfg 5's gap between the jittered bench (previous step's iteration counts as the
dispatch prediction) and a repeated batch (exact prediction) the prediction, or something else?
Per step: (a) the bench protocol (setup + warm start + solve, order from the previous step);
(b) the same step's batch solved again right after (order from its own counts: exact).
Prints the solve-call times (HIP-synchronised wall clock) of both.
  python3 tools/order_probe.py [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "python-mpc_amd"), ROOT]
import numpy as np  # noqa: E402


def main():
    import torch
    import bench
    from osqp_amd import DeviceBatch, _drop_common_zeros
    from osqp_amd.mpc_device import warm_shift
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    cfg, B = 5, 8192
    dev = torch.device("cuda", 0)
    b = bench.make_shard(cfg, B, 1, 0)
    P, Px = _drop_common_zeros(b["P"], b["Px"])
    A, Ax = _drop_common_zeros(b["A"], b["Ax"])
    s = {k: v for k, v in b["settings"].items() if k != "verbose"}
    to_dev = lambda a, dtype=torch.float64: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dtype=dtype).contiguous()  # noqa: E731
    dPx, dAx, dq = (to_dev(a) for a in (Px, Ax, b["q"]))
    seq = bench.bound_sequence(b, steps + 1, bench.instance_seed(cfg, 0), to_dev)
    dx = torch.empty((B, b["n"]), dtype=torch.float64, device=dev)
    dy = torch.empty((B, b["m"]), dtype=torch.float64, device=dev)
    dst = torch.empty(B, dtype=torch.int32, device=dev)
    dit = torch.empty(B, dtype=torch.int32, device=dev)
    h = DeviceBatch(P, A, B, device=0, **s)
    h.setup(dPx, dAx, dq, *seq[0])
    h.solve(dx, dy, dst, dit)
    h.synchronize()
    xs, ys = warm_shift(b["N"], 8, 2, dx, dy)
    torch.cuda.synchronize()

    def run(t):
        h.setup(dPx, dAx, dq, *seq[t])
        h.warm_start(xs, ys)
        h.synchronize()
        t0 = time.perf_counter()
        h.solve(dx, dy, dst, dit)
        h.synchronize()
        return (time.perf_counter() - t0) * 1e3

    a, e = [], []
    for t in range(1, steps + 1):
        a.append(run(t))   # order from step t-1's counts
        e.append(run(t))   # order from step t's own counts
    print("previous-step order: solve ms", np.round(a, 2).tolist(), "mean", round(float(np.mean(a[1:])), 3))
    print("exact order:         solve ms", np.round(e, 2).tolist(), "mean", round(float(np.mean(e[1:])), 3))


if __name__ == "__main__":
    main()
