#!/usr/bin/env python3
"""Diagnostic (phase-timer build, MPCQP_PHASE_PROF=1): the real dispatch timeline of the cfg-5
long-horizon kernel -- per instance its start (100 MHz wall clock), duration and CU -- for the
bench protocol's order (the previous step's counts) and for the exact order (the same batch
solved again).  Prints per-CU busy / idle figures and the makespan structure.
  MPCQP_PHASE_PROF=1 python3 tools/dispatch_timeline.py [out.npz]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "python-mpc_amd"), ROOT]
os.environ.setdefault("MPCQP_PHASE_PROF", "1")
import numpy as np  # noqa: E402


def main():
    import torch
    import bench
    from osqp_amd import DeviceBatch, _drop_common_zeros
    from osqp_amd.mpc_device import warm_shift
    cfg, B = 5, 8192
    dev = torch.device("cuda", 0)
    b = bench.make_shard(cfg, B, 1, 0)
    P, Px = _drop_common_zeros(b["P"], b["Px"])
    A, Ax = _drop_common_zeros(b["A"], b["Ax"])
    s = {k: v for k, v in b["settings"].items() if k != "verbose"}
    to_dev = lambda a, dtype=torch.float64: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dtype=dtype).contiguous()  # noqa: E731
    dPx, dAx, dq = (to_dev(a) for a in (Px, Ax, b["q"]))
    seq = bench.bound_sequence(b, 5, bench.instance_seed(cfg, 0), to_dev)
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
    out = {}

    def run(t, tag):
        h.setup(dPx, dAx, dq, *seq[t])
        h.warm_start(xs, ys)
        h.solve(dx, dy, dst, dit)
        h.synchronize()
        pt = h.phase_times()
        st, du = pt[:, 15], pt[:, 7]
        cu = (pt[:, 23] & 15) * 65536 + ((pt[:, 22] >> 8) & 0xFFF)
        st = st - st.min()
        end = st + du
        ms = end.max() * 1e-5
        cus = np.unique(cu)
        busy = np.array([du[cu == c].sum() for c in cus])
        last_end = np.array([end[cu == c].max() for c in cus])
        nper = np.array([(cu == c).sum() for c in cus])
        print(f"{tag}: makespan {ms:.2f} ms, {len(cus)} CUs, instances per CU {nper.min()}-{nper.max()}, "
              f"CU busy mean {busy.mean() * 1e-5:.2f} ms (max {busy.max() * 1e-5:.2f}), CU last end p10 "
              f"{np.percentile(last_end, 10) * 1e-5:.2f} p50 {np.percentile(last_end, 50) * 1e-5:.2f} ms")
        # gaps: per CU, start of each instance minus the end of the previous one on that CU
        gaps = []
        for c in cus:
            sel = np.argsort(st[cu == c])
            s_, e_ = st[cu == c][sel], end[cu == c][sel]
            gaps.extend((s_[1:] - e_[:-1]).tolist())
        gaps = np.array(gaps) * 1e-2
        print(f"   gaps between instances on a CU (us): mean {gaps.mean():.1f} p99 {np.percentile(gaps, 99):.1f} "
              f"max {gaps.max():.1f}; last-started instance at {st.max() * 1e-5:.2f} ms, longest {du.max() * 1e-5:.2f} ms "
              f"started at {st[np.argmax(du)] * 1e-5:.2f} ms")
        late = np.argsort(-end)[:5]
        print("   last to end: start ms", np.round(st[late] * 1e-5, 2).tolist(), "dur ms", np.round(du[late] * 1e-5, 2).tolist(),
              "iters", dit.cpu().numpy()[late].tolist())
        out[tag] = np.stack([st, du, cu, dit.cpu().numpy()])

    for t in (1, 2, 3):
        run(t, f"step{t} prev-order")
        run(t, f"step{t} exact-order")
    if len(sys.argv) > 1:
        np.savez_compressed(sys.argv[1], **out)


if __name__ == "__main__":
    main()
