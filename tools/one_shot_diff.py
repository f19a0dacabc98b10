"""Diagnostic: where the one-shot fused kernel's outputs differ from the persisting kernel's
(and whether two persisting handles agree bit for bit).  python3 tools/one_shot_diff.py [cfg] [B]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "python-mpc_amd"))
from test_one_shot import _inputs, _out  # noqa: E402
from osqp_amd import DeviceBatch  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
dev = torch.device("cuda", 0)
P, A, s, (Px, Ax, q), bounds, b = _inputs(cfg, B, 31, dev)
hs = [DeviceBatch(P, A, B, device=0, **s) for _ in range(4)]
print("one-shot applies:", hs[2].one_shot(True), hs[3].one_shot(True))
l, u = bounds[0]
outs = []
for h in hs:
    o = _out(B, b["n"], b["m"], dev)
    h.setup_solve(Px, Ax, q, l, u, *o)
    torch.cuda.synchronize()
    outs.append([t.cpu().numpy() for t in o])


def cmp(i, j):
    x1, y1, s1, it1 = outs[i]
    x2, y2, s2, it2 = outs[j]
    dx = ~((x1.view(np.int64) == x2.view(np.int64)).all(1))
    dy = ~((y1.view(np.int64) == y2.view(np.int64)).all(1))
    rows = np.nonzero(dx | dy)[0]
    print(f"handles {i} vs {j}: x rows differ {dx.sum()}, y rows {dy.sum()}, status differ {(s1 != s2).sum()}, "
          f"iters differ {(it1 != it2).sum()}")
    if len(rows):
        r = rows[:10]
        print("  rows", r.tolist(), "status", s1[r].tolist(), s2[r].tolist(), "iters", it1[r].tolist(), it2[r].tolist())
        print("  max |dx|", np.nanmax(np.abs(x1[rows] - x2[rows])), "nan x1/x2", np.isnan(x1).any(1).sum(),
              np.isnan(x2).any(1).sum())
        k = rows[0]
        c = np.nonzero(x1[k].view(np.int64) != x2[k].view(np.int64))[0]
        print("  row", k, "cols", c[:12].tolist(), x1[k, c[:4]].tolist(), x2[k, c[:4]].tolist())


cmp(0, 1)
cmp(2, 3)
cmp(0, 2)
print("status counts", np.unique(outs[0][2], return_counts=True), "iters", outs[0][3].min(), outs[0][3].max())
