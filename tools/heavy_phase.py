#!/usr/bin/env python3
"""Diagnostic: the phase breakdown (in-kernel timers, MPCQP_PHASE_PROF=1) of the heaviest cfg-2
bench instance solved ALONE (B = 1) -- the instance whose latency sets the headline launch.
  python tools/heavy_phase.py [rank]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "python-mpc_amd"), os.path.join(ROOT, "oracle"), ROOT]
os.environ.setdefault("MPCQP_PHASE_PROF", "1")
import numpy as np  # noqa: E402


def main():
    import torch
    import bench
    import pyoracle
    from osqp_amd import DeviceBatch, _drop_common_zeros
    b = bench.make_shard(2, 1024, 1, 0)
    P, Px = _drop_common_zeros(b["P"], b["Px"])
    A, Ax = _drop_common_zeros(b["A"], b["Ax"])
    s = {k: v for k, v in b["settings"].items() if k != "verbose"}
    ro = pyoracle.solve_batch(P, A, Px, b["q"], Ax, b["l"], b["u"], nthreads=16, **s)
    k = int(np.argsort(-ro.iter, kind="stable")[int(sys.argv[1]) if len(sys.argv) > 1 else 0])
    dev = torch.device("cuda", 0)
    put = lambda a: torch.from_numpy(np.ascontiguousarray(a[k:k + 1])).to(dev)  # noqa: E731
    X = [put(Px), put(Ax), put(b["q"]), put(b["l"]), put(b["u"])]
    o = [torch.empty((1, b["n"]), dtype=torch.float64, device=dev), torch.empty((1, b["m"]), dtype=torch.float64, device=dev),
         torch.empty(1, dtype=torch.int32, device=dev), torch.empty(1, dtype=torch.int32, device=dev)]
    h = DeviceBatch(P, A, 1, device=0, **s)
    for _ in range(3):
        h.setup(*X)
        h.solve(*o)
    h.synchronize()
    h.timing(True)
    h.setup(*X)
    h.solve(*o)
    kt = h.timing_read()
    pt = h.phase_times().astype(np.float64)[0]
    it = int(o[3].cpu().item())
    names = ["factor", "rhs", "bt_solve", "update", "checks", "tail"]
    print(f"instance {k} (oracle iters {ro.iter[k]}, rho updates {getattr(ro, 'rho_updates', [None] * 1024)[k]}) "
          f"alone: iters {it}, solve kernel {kt['solve_ms']:.3f} ms, {pt[6]:.0f} cyc = {pt[7] * 1e-2:.1f} us, "
          f"{pt[6] / max(it, 1):.0f} cyc/iter")
    for j, nm in enumerate(names):
        print(f"   {nm:9s} {pt[j]:10.0f} cyc {100 * pt[j] / pt[6]:5.1f}%  {pt[j] / max(it, 1):7.0f} /iter")
    for j, nm in zip(range(8, 15), ["f.asm", "f.F/S", "f.GJ", "f.epi", "s.A", "s.B", "s.C"]):
        print(f"     {nm:7s} {pt[j]:10.0f} cyc")


if __name__ == "__main__":
    main()
