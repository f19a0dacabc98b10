#!/usr/bin/env python3
"""Offline study of the dispatch-order predictor on traced iteration counts (tools/pred_trace.py):
list scheduling of each step's instances on `slots` workgroup slots in the order a predictor
gives, duration = iterations + a per-instance constant; makespan relative to the exact-order one.
  python3 tools/pred_sim.py trace.npz [slots] [const_iters]"""
import heapq
import sys

import numpy as np


def makespan(dur, order, slots):
    h = [0.0] * slots
    for i in order:
        t = heapq.heappop(h)
        heapq.heappush(h, t + dur[i])
    return max(h)


def lpt(key):
    # counting sort on key >> 4 descending, stable by index (kernels.hip::k_order)
    k = np.minimum(key >> 4, 255)
    return np.lexsort((np.arange(len(key)), -k))


def main():
    d = np.load(sys.argv[1])
    it = d["iters"].astype(np.int64)
    slots = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    c = float(sys.argv[3]) if len(sys.argv) > 3 else 10.0
    S, B = it.shape
    res = {}
    preds = {
        "identity": lambda t, st: np.zeros(B, np.int64),
        "previous (current)": lambda t, st: it[t - 1],
        "exact": lambda t, st: it[t],
    }
    for dec in (0.5, 0.75, 0.9):
        preds[f"max-decay {dec}"] = (lambda dec: lambda t, st: st.setdefault(dec, None))(dec)
    for name in preds:
        tot = []
        state = None
        for t in range(1, S):
            if name.startswith("max-decay"):
                dec = float(name.split()[1])
                if state is None:
                    state = it[0].astype(np.float64)
                key = np.maximum(it[t - 1], np.floor(state)).astype(np.int64)
                state = np.maximum(it[t - 1].astype(np.float64), dec * state)
            else:
                key = preds[name](t, None)
            order = np.arange(B) if name == "identity" else lpt(key)
            tot.append(makespan(it[t] + c, order, slots))
        res[name] = np.mean(tot[2:])  # (after the predictor's warm-up)
    base = res["exact"]
    ideal = np.mean([(it[t] + c).sum() / slots for t in range(3, S)])
    for k, v in res.items():
        print(f"{k:22s} makespan {v:9.0f} iteration-units  x{v / base:.3f} of exact  (ideal {ideal / v:.3f})")
    chg = np.abs(np.diff(it, axis=0))
    print("step-to-step |d iters|: mean", chg.mean().round(1), "p99", np.percentile(chg, 99), "max", chg.max(),
          "; iters mean", it.mean().round(1), "max", it.max())


if __name__ == "__main__":
    main()
