"""Diagnostic: the batch setup's time per call against the batch size (cfg 5 default), to tell
a latency-bound setup kernel (time flat until the CUs fill) from a throughput-bound one.
  MPCQP_PKG=<pkg dir> python3 tools/setup_scan.py [cfg] [B ...]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("MPCQP_PKG", os.path.join(ROOT, "python-mpc_amd")))
import torch  # noqa: E402
from osqp_amd import DeviceBatch, mpc, _drop_common_zeros  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 5
Bs = [int(a) for a in sys.argv[2:]] or [1, 256, 512, 1024, 2048, 4096, 8192]
b0 = mpc.make_batch(cfg, B=max(Bs), seed=5)
P, Px = _drop_common_zeros(b0["P"], b0["Px"])
A, Ax = _drop_common_zeros(b0["A"], b0["Ax"])
s = {k: v for k, v in b0["settings"].items() if k != "verbose"}
if os.environ.get("SCAN_SCALING"):  # the Ruiz pass count (10 by default): the per-pass cost
    s["scaling"] = int(os.environ["SCAN_SCALING"])
dev = torch.device("cuda", 0)
t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
D = [t(a) for a in (Px, Ax, b0["q"], b0["l"], b0["u"])]
for B in Bs:
    h = DeviceBatch(P, A, B, device=0, **s)
    args = [d[:B] for d in D]
    for _ in range(3):
        h.setup(*args)
    h.synchronize()
    k = 20
    t0 = time.perf_counter()
    for _ in range(k):
        h.setup(*args)
    h.synchronize()
    ms = (time.perf_counter() - t0) / k * 1e3
    print(f"cfg {cfg} scaling {s.get('scaling', 10)} B {B:6d} setup {ms:8.3f} ms  {ms * 1e3 / B:8.3f} us/instance", flush=True)
    del h
