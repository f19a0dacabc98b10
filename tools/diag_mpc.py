"""Diagnostic (GPU): one DynamicMPC step, statuses and the host-API solve of the same QP."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "python-mpc_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np
import torch
from osqp_amd import OSQP, mpc
from osqp_amd.mpc_device import DynamicMPC
from test_mpc_device import path

B, N = 4, int(sys.argv[1]) if len(sys.argv) > 1 else 30
x0 = np.zeros((B, 6)); x0[:, 3] = 15.0
x0[:, 1] = [0.0, 1.0, -1.5, 0.5]; x0[:, 2] = np.deg2rad([0.0, 5.0, -3.0, 10.0])
px, py = path()
ctl = DynamicMPC(x0, np.zeros((B, 2)), px, py, N=N)
print("plan", ctl.solver.plan_info())
for k in range(8):
    xt = ctl.xt.cpu().numpy()
    st, it = ctl.step()
    torch.cuda.synchronize()
    print("step", k, "status", st.cpu().numpy(), "iters", it.cpu().numpy(), "xt", xt[:, :4].round(3).tolist())
    if (st.cpu().numpy() != 1).any():
        break
last = {k: v.cpu().numpy() for k, v in ctl.last.items()}
print("l>u", (last["l"] > last["u"]).sum(), "nonfinite q", (~np.isfinite(last["q"])).sum(),
      "nonfinite Ax", (~np.isfinite(last["Ax"])).sum(), "Px", ctl.Px[0, :8].cpu().numpy())
P, A, _, _ = ctl.layout.pattern()
for b in range(B):
    A.data = last["Ax"][b]
    g = OSQP(); g.setup(P, last["q"][b], A, last["l"][b], last["u"][b], polish=False, warm_start=False)
    r = g.solve(); print("host-API", b, r.info.status, r.info.iter)
    import pyoracle
    o = pyoracle.OSQP(); o.setup(P, last["q"][b], A, last["l"][b], last["u"][b], polish=False, warm_start=False)
    r = o.solve(); print("oracle", b, r.info.status, r.info.iter)
