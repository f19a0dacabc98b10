#!/usr/bin/env python3
"""Diagnostic: how fast do the predicted-heaviest cfg-2 instances run ALONE on a CU?

The cfg-2 bench batch (bench.make_shard(2, 1024)) is solved by the oracle on the host to rank its
instances by iteration count; the top H are then solved on the device as a batch of their own
(H workgroups: at most one per CU), and the full batch beside it.  Prints ms per fused
setup+solve launch (HIP events, the median of `reps`).  Run under MPCQP_BUILD=exp
MPCQP_DENSE_W4=1 for the dense-inverse form."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "python-mpc_amd"), os.path.join(ROOT, "oracle"), ROOT]
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
    rank = np.argsort(-ro.iter, kind="stable")
    dev = torch.device("cuda", 0)
    out = {"build": os.environ.get("MPCQP_BUILD", ""), "dense": os.environ.get("MPCQP_DENSE_W4", "")}
    for H in [int(v) for v in (sys.argv[1:] or ["1", "8", "32", "1024"])]:
        idx = rank[:H] if H < 1024 else np.arange(1024)
        put = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        X = [put(Px[idx]), put(Ax[idx]), put(b["q"][idx]), put(b["l"][idx]), put(b["u"][idx])]
        o = [torch.empty((H, b["n"]), dtype=torch.float64, device=dev),
             torch.empty((H, b["m"]), dtype=torch.float64, device=dev),
             torch.empty(H, dtype=torch.int32, device=dev), torch.empty(H, dtype=torch.int32, device=dev)]
        h = DeviceBatch(P, A, H, device=0, **s)
        st = torch.cuda.ExternalStream(h.stream_handle().value, device=dev)
        ts = []
        for r in range(13):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            h.setup_solve(*X, *o)
            e1.record(st)
            h.synchronize()
            if r >= 3:
                ts.append(e0.elapsed_time(e1))
        it = o[3].cpu().numpy()
        out[f"H{H}"] = {"ms": float(np.median(ts)), "iters_max": int(it.max()), "iters_oracle_max": int(ro.iter[idx].max()),
                        "iter_match": float(np.mean(it == ro.iter[idx])), "variant": h.plan_info()["variant"]}
        del h
    print(json.dumps(out))


if __name__ == "__main__":
    main()
