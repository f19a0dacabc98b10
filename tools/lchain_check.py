"""Diagnostic: outputs of a batch (cold setup + solve, then a warm-started solve; on cfg 2 / 3
also the one-shot fused setup + solve) for a bit-for-bit A/B of two builds or two settings.
  MPCQP_PKG=<pkg dir> python3 tools/lchain_check.py out.npz [B] [cfg, default 5]
  python3 tools/lchain_check.py --compare a.npz b.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if sys.argv[1] == "--compare":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    for k in a.files:
        same = np.array_equal(a[k].view(np.int64) if a[k].dtype == np.float64 else a[k],
                              b[k].view(np.int64) if b[k].dtype == np.float64 else b[k])
        print(k, "bit-identical" if same else f"DIFFER max {np.nanmax(np.abs(a[k] - b[k]))}")
    sys.exit(0)
sys.path.insert(0, os.environ.get("MPCQP_PKG", os.path.join(ROOT, "python-mpc_amd")))
import torch  # noqa: E402
from osqp_amd import DeviceBatch, mpc, _drop_common_zeros  # noqa: E402

B = int(sys.argv[2]) if len(sys.argv) > 2 else 512
cfg = int(sys.argv[3]) if len(sys.argv) > 3 else 5
b = mpc.make_batch(cfg, B=B, seed=77)
P, Px = _drop_common_zeros(b["P"], b["Px"])
A, Ax = _drop_common_zeros(b["A"], b["Ax"])
s = {k: v for k, v in b["settings"].items() if k != "verbose"}
dev = torch.device("cuda", 0)
t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
dPx, dAx, dq, dl, du = (t(a) for a in (Px, Ax, b["q"], b["l"], b["u"]))
torch.cuda.synchronize()
h = DeviceBatch(P, A, B, device=0, **s)
out = {}
if cfg != 5 and hasattr(h, "one_shot"):  # the fused setup + solve, one-shot form, too
    h1 = DeviceBatch(P, A, B, device=0, **s)
    h1.one_shot(True)
    o = [torch.empty((B, b["n"]), dtype=torch.float64, device=dev), torch.empty((B, b["m"]), dtype=torch.float64, device=dev),
         torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.int32, device=dev)]
    h1.setup_solve(dPx, dAx, dq, dl, du, *o)
    h1.synchronize()
    out.update({f"one_{k}": v.cpu().numpy() for k, v in zip(("x", "y", "st", "it"), o)})
for tag in ("cold", "warm"):
    x = torch.empty((B, b["n"]), dtype=torch.float64, device=dev)
    y = torch.empty((B, b["m"]), dtype=torch.float64, device=dev)
    st = torch.empty(B, dtype=torch.int32, device=dev)
    it = torch.empty(B, dtype=torch.int32, device=dev)
    if tag == "cold":
        h.setup(dPx, dAx, dq, dl, du)
    else:
        h.update(q=dq * 1.01)
    h.solve(x, y, st, it)
    h.synchronize()
    out.update({f"{tag}_x": x.cpu().numpy(), f"{tag}_y": y.cpu().numpy(), f"{tag}_st": st.cpu().numpy(),
                f"{tag}_it": it.cpu().numpy()})
if cfg == 5:  # setup + warm start from the cold solution (fused where the build has it)
    h2 = DeviceBatch(P, A, B, device=0, **s)
    o = [torch.empty((B, b["n"]), dtype=torch.float64, device=dev), torch.empty((B, b["m"]), dtype=torch.float64, device=dev),
         torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.int32, device=dev)]
    x0, y0 = (torch.from_numpy(out[k]).to(dev) for k in ("cold_x", "cold_y"))
    if hasattr(h2, "setup_warm") and os.environ.get("LCHAIN_FUSED_WARM", "1") == "1":
        h2.setup_warm(dPx, dAx, dq * 1.01, dl, du, x0, y0)
    else:
        h2.setup(dPx, dAx, dq * 1.01, dl, du)
        h2.warm_start(x0, y0)
    h2.solve(*o)
    h2.synchronize()
    out.update({f"sw_{k}": v.cpu().numpy() for k, v in zip(("x", "y", "st", "it"), o)})
np.savez(sys.argv[1], **out)
print("saved", sys.argv[1], "solved", float((out["cold_st"] == 1).mean()), "iters", out["cold_it"].mean())
