#!/usr/bin/env python3
"""Phase breakdown of k_solve from the in-kernel timers (diagnostic, GPU only).

  MPCQP_PHASE_PROF=1 python tools/phase_prof.py --config 2 [--batch B]

Prints, for the slowest instance and for the mean instance, cycles per phase
(factor, rhs, bt_solve, update, checks, tail) and cycles per ADMM iteration.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_pkg = [a.split("=", 1)[1] for a in sys.argv if a.startswith("--pkg=")]  # A/B: another build's package
sys.path.insert(0, _pkg[0] if _pkg else os.path.join(ROOT, "python-mpc_amd"))
os.environ.setdefault("MPCQP_PHASE_PROF", "1")

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--pkg", default=None, help="package directory of another build (--pkg=DIR)")
    args = ap.parse_args()
    import torch
    from osqp_amd import DeviceBatch, mpc, _drop_common_zeros
    spec = mpc.CONFIGS[args.config]
    B = args.batch or spec["B"]
    b = mpc.make_batch(args.config, B=B, seed=1000 * args.config)
    P, Px = _drop_common_zeros(b["P"], b["Px"])
    A, Ax = _drop_common_zeros(b["A"], b["Ax"])
    settings = {k: v for k, v in b["settings"].items() if k != "verbose"}
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    dPx, dAx, dq, dl, du = (t(a) for a in (Px, Ax, b["q"], b["l"], b["u"]))
    dx = torch.empty((B, b["n"]), dtype=torch.float64, device=dev)
    dy = torch.empty((B, b["m"]), dtype=torch.float64, device=dev)
    dst = torch.empty(B, dtype=torch.int32, device=dev)
    dit = torch.empty(B, dtype=torch.int32, device=dev)
    s = DeviceBatch(P, A, B, device=0, **settings)
    for _ in range(3):
        s.setup(dPx, dAx, dq, dl, du)
        s.solve(dx, dy, dst, dit)
    s.synchronize()
    s.timing(True)
    s.setup(dPx, dAx, dq, dl, du)
    s.solve(dx, dy, dst, dit)
    kt = s.timing_read()
    pt = s.phase_times().astype(np.float64)
    it = dit.cpu().numpy().astype(np.float64)
    names = ["factor", "rhs", "bt_solve", "update", "checks", "tail"]
    if B == 1:  # the oracle's rho-update count: factorisations = 1 + updates (the first one may be setup()'s)
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle
        o = pyoracle.OSQP()
        Pk, Ak = P.copy(), A.copy()
        Pk.data, Ak.data = Px[0].copy(), Ax[0].copy()
        o.setup(Pk, b["q"][0], Ak, b["l"][0], b["u"][0], **settings)
        r = o.solve()
        print(f"oracle: iters {r.info.iter}, rho updates {r.info.rho_updates}")
    print(f"config {args.config} B={B} plan={s.plan_info()} kernel_ms={kt['solve_ms']:.3f}")
    slow = int(np.argmax(pt[:, 7]))
    if pt[:, 15].any():  # absolute start stamps (two-wave kernel): residency rounds and the critical instance
        st = pt[:, 15] - pt[:, 15].min()
        end = st + pt[:, 7]
        last = int(np.argmax(end))
        q = np.percentile(st, [50, 75, 90, 100]) * 1e-2
        print(f"starts (us after the first): p50 {q[0]:.1f} p75 {q[1]:.1f} p90 {q[2]:.1f} max {q[3]:.1f}; "
              f"started within 2 us: {int((st < 200).sum())} of {len(st)}")
        print(f"last to finish: instance {last} started {st[last] * 1e-2:.1f} us, ran {pt[last, 7] * 1e-2:.1f} us, "
              f"iters {it[last]:.0f}; span {end.max() * 1e-2:.1f} us")
    for label, row, its in (("slowest", pt[slow], it[slow]), ("mean", pt.mean(0), it.mean())):
        tot = row[6]
        mhz = row[6] / (row[7] * 10e-3) if row[7] else 0
        print(f"{label}: iters {its:.1f} total {tot:.0f} cyc = {row[7] * 1e-2:.1f} us  (~{mhz:.0f} MHz shader clock)"
              f"  {tot / max(its, 1):.0f} cyc/iter")
        for k, nm in enumerate(names):
            print(f"   {nm:9s} {row[k]:12.0f} cyc {100 * row[k] / tot:5.1f}%  {row[k] / max(its, 1):8.0f} /iter")
        for k, nm in zip(range(8, 12), ["f.asm", "f.F/S", "f.GJ", "f.epi"]):
            print(f"     {nm:7s} {row[k]:12.0f} cyc")
        if row[12:15].any():
            for k, nm in zip(range(12, 15), ["s.A", "s.B", "s.C"]):
                print(f"     {nm:7s} {row[k]:12.0f} cyc  {row[k] / max(its, 1):8.0f} /iter")
        if row.size > 16 and row[16:24].any():  # the long-horizon interface form's own per-wave times
            for k, nm in zip(range(16, 22), ["fwd.top", "fwd.bot", "bwd.top", "bwd.bot", "T.w0", "X.w0"]):
                print(f"     {nm:7s} {row[k]:12.0f} cyc  {row[k] / max(its, 1):8.0f} /iter (own)")


if __name__ == "__main__":
    main()
