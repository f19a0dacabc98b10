"""Diagnostic: the wide batch setup's forms (512 / 1024 threads, MPCQP_SETUP_FULL) and the fused
setup + warm start against setup() + warm_start(), cfg 5: which combinations agree bit for bit.
  python3 tools/wide_forms_check.py [B]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-mpc_amd"))
import torch  # noqa: E402
from osqp_amd import DeviceBatch, mpc, _drop_common_zeros  # noqa: E402
from osqp_amd.mpc_device import warm_shift  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 640
b = mpc.make_batch(5, B=B, seed=41)
P, Px = _drop_common_zeros(b["P"], b["Px"])
A, Ax = _drop_common_zeros(b["A"], b["Ax"])
s = {k: v for k, v in b["settings"].items() if k != "verbose"}
dev = torch.device("cuda", 0)
t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
dPx, dAx, dq, dl, du = (t(a) for a in (Px, Ax, b["q"], b["l"], b["u"]))


def outs():
    return (torch.empty((B, b["n"]), dtype=torch.float64, device=dev),
            torch.empty((B, b["m"]), dtype=torch.float64, device=dev),
            torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.int32, device=dev))


def same(a, c):
    return np.array_equal(a.view(np.int64) if a.dtype == np.float64 else a, c.view(np.int64) if c.dtype == np.float64 else c)


res = {}
for full in ("0", "1"):
    os.environ["MPCQP_SETUP_FULL"] = full
    h = DeviceBatch(P, A, B, device=0, **s)
    o = outs()
    h.setup(dPx, dAx, dq, dl, du)
    h.solve(*o)
    h.synchronize()
    res[("cold", full)] = [v.cpu().numpy() for v in o]
    if full == "0":
        xs, ys = warm_shift(b["N"], 8, 2, o[0], o[1])
        torch.cuda.synchronize()
    for yk, y0 in (("y", ys), ("noy", None)):
        for fused in (False, True):
            h = DeviceBatch(P, A, B, device=0, **s)
            o = outs()
            if fused:
                h.setup_warm(dPx, dAx, dq, dl, du, xs, y0)
            else:
                h.setup(dPx, dAx, dq, dl, du)
                h.warm_start(xs, y0)
            h.solve(*o)
            h.synchronize()
            res[(yk, full, fused)] = [v.cpu().numpy() for v in o]
for k, v in res.items():
    print(k, "solved", float((v[2] == 1).mean()), "iters", float(v[3].mean()))
ref = res[("cold", "0")]
print("cold full vs half:", [same(a, c) for a, c in zip(ref, res[("cold", "1")])])
for yk in ("y", "noy"):
    r0 = res[(yk, "0", False)]
    for k in [(yk, "0", True), (yk, "1", False), (yk, "1", True)]:
        print(yk, "half-separate vs", k, [same(a, c) for a, c in zip(r0, res[k])])
