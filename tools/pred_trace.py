#!/usr/bin/env python3
"""Diagnostic: per-step iteration counts of the bench protocol (a distinct jittered batch each
step, cfg 5 warm-started as bench.py runs it), for offline study of the dispatch-order
predictor (tools/pred_sim.py).  Writes an npz of iters[step, instance] and the kernel ms.
  python3 tools/pred_trace.py out.npz [config] [steps] [batch]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "python-mpc_amd"), ROOT]
import numpy as np  # noqa: E402


def main():
    import torch
    import bench
    from osqp_amd import DeviceBatch, mpc, _drop_common_zeros
    out = sys.argv[1]
    cfg = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    B = int(sys.argv[4]) if len(sys.argv) > 4 else mpc.CONFIGS[cfg]["B"]
    dev = torch.device("cuda", 0)
    b = bench.make_shard(cfg, B, 1, 0)
    P, Px = _drop_common_zeros(b["P"], b["Px"])
    A, Ax = _drop_common_zeros(b["A"], b["Ax"])
    s = {k: v for k, v in b["settings"].items() if k != "verbose"}
    to_dev = lambda a, dtype=torch.float64: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dtype=dtype).contiguous()  # noqa: E731
    dPx, dAx, dq = (to_dev(a) for a in (Px, Ax, b["q"]))
    seq = bench.bound_sequence(b, steps + 1, bench.instance_seed(cfg, 0), to_dev,
                               jitter=float(os.environ.get("MPCQP_TRACE_JITTER", bench.JITTER)))
    n, m = b["n"], b["m"]
    dx = torch.empty((B, n), dtype=torch.float64, device=dev)
    dy = torch.empty((B, m), dtype=torch.float64, device=dev)
    dst = torch.empty(B, dtype=torch.int32, device=dev)
    dit = torch.empty(B, dtype=torch.int32, device=dev)
    h = DeviceBatch(P, A, B, device=0, **s)
    warm = cfg == 5
    xs = ys = None
    if warm:
        from osqp_amd.mpc_device import warm_shift
        h.setup(dPx, dAx, dq, *seq[0])
        h.solve(dx, dy, dst, dit)
        h.synchronize()
        xs, ys = warm_shift(b["N"], 8, 2, dx, dy)
    torch.cuda.synchronize()
    its, ms, rus, cyc = [], [], [], []
    import ctypes as C
    from osqp_amd import lib
    prof = os.environ.get("MPCQP_PHASE_PROF") == "1"
    for t in range(steps + 1):
        t0 = time.perf_counter()
        if warm:
            h.setup(dPx, dAx, dq, *seq[t])
            h.warm_start(xs, ys)
            h.solve(dx, dy, dst, dit)
        else:
            h.setup_solve(dPx, dAx, dq, *seq[t], dx, dy, dst, dit)
        h.synchronize()
        ms.append((time.perf_counter() - t0) * 1e3)
        its.append(dit.cpu().numpy().copy())
        ru = np.zeros(B, np.int32)
        f = np.zeros(B)
        dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
        lib().mpcqp_get_info_batch(h._h.ptr, dp(f), dp(f), dp(f), dp(f), ru.ctypes.data_as(C.POINTER(C.c_int32)))
        rus.append(ru)
        if prof:  # per-instance solve cycles (the phase-timer build's total slot)
            cyc.append(h.phase_times()[:, 6].astype(np.int64))
    np.savez_compressed(out, iters=np.array(its), ms=np.array(ms), rho_upd=np.array(rus),
                        cycles=np.array(cyc) if cyc else np.zeros((0, B), np.int64))
    print("steps", len(its), "ms", np.round(ms, 2).tolist())


if __name__ == "__main__":
    main()
