#!/usr/bin/env python3
"""LDS bank-conflict model of the four-wave kernel's per-iteration gathers (CPU only).

MI355X_MICROARCH.md (LDS): ds_read_b64 serves a wave64 in two lane groups of 32, one LDS
cycle per group when conflict-free, bank of byte address a = (a / 4) mod 64; each extra
distinct address on a busy bank adds a cycle.  This replays the gathers of one ADMM iteration
on a layout (cfg 2 by default) from the plan's padded column order: the rows phase (lane =
row i reads x~ at the k-th column of its row) and the rhs (lane = padded column reads w at the
k-th row of its column), 8-byte values at base + 8 * index, and reports the LDS cycles per
list position against the conflict-free two.  With --swizzle the model stores index v at
v + (v >> 5) (one pad slot per 32 values) to show what a padded layout would change.

  python tools/lds_banks.py [--config 2] [--swizzle]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-mpc_amd"))

import numpy as np  # noqa: E402


def cycles(addrs):
    """LDS cycles of one ds_read_b64 over the 64 lanes' byte addresses (None: inactive lane)."""
    total = 0
    for g in (range(0, 32), range(32, 64)):
        banks = {}
        for ln in g:
            a = addrs[ln]
            if a is None:
                continue
            for dw in (a // 4, a // 4 + 1):
                banks.setdefault(dw % 64, set()).add(a)
        total += max([len(v) for v in banks.values()] or [1])
    return total


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--swizzle", action="store_true")
    a = ap.parse_args()
    from osqp_amd import analyze, canonical_data, mpc
    b = mpc.make_batch(a.config, B=1, seed=1)
    P, A = canonical_data(b["P"], b["A"])
    nb, blk, var_pad, _ = analyze(P, A)
    A = A.tocsr()
    m, n = A.shape
    pos = (lambda v: v + (v >> 5)) if a.swizzle else (lambda v: v)
    rows = [[int(var_pad[j]) for j in A.indices[A.indptr[i]:A.indptr[i + 1]]] for i in range(m)]
    Ac = A.tocsc()
    pad_of = {int(var_pad[j]): j for j in range(n)}
    npad = nb * blk
    cols = [[int(r) for r in Ac.indices[Ac.indptr[pad_of[pc]]:Ac.indptr[pad_of[pc] + 1]]] if pc in pad_of else []
            for pc in range(npad)]

    def phase(lists, nlanes, name):
        K = max(len(x) for x in lists)
        tot = ideal = 0
        for w0 in range(0, nlanes, 64):
            for k in range(K):
                addrs = [8 * pos(lists[i][k]) if i < len(lists) and k < len(lists[i]) else None
                         for i in range(w0, w0 + 64)]
                if all(x is None for x in addrs):
                    continue
                tot += cycles(addrs)
                ideal += 2
        print(f"{name}: {tot} LDS cycles over the waves' {K}-deep gathers, conflict-free {ideal} "
              f"({tot / max(ideal, 1):.2f}x)")

    print(f"config {a.config}: n={n} m={m} nb={nb} npad={npad}{' (swizzled layout)' if a.swizzle else ''}")
    # S-tile loads (Gauss-Jordan register load, run-start SB load): lane (h, i) reads row i,
    # columns [16 h + jj, +2) of a row-major 32 x 32 tile with ds_read_b128 -- lane groups of
    # 16 (MI355X_MICROARCH.md); with --swizzle the column pair index is XORed with (i & 7)
    groups = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
              list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
    groups += [[g + 32 for g in x] for x in groups]
    tot = 0
    for jj in range(0, 16, 2):
        for grp in groups:
            banks = {}
            for ln in grp:
                i, h = ln & 31, ln >> 5
                c = 16 * h + ((jj ^ (2 * (i & 7))) if a.swizzle else jj)
                addr = 8 * (i * 32 + c)
                for dw in range(addr // 4, addr // 4 + 4):
                    banks.setdefault(dw % 64, set()).add(addr)
            tot += max(len(v) for v in banks.values())
    print(f"S-tile load of one wave (8 x ds_read_b128): {tot} LDS cycles, conflict-free 32 ({tot / 32:.0f}x)")
    phase(rows, m, "rows phase, x~ at the row's columns")
    phase(cols, npad, "rhs, w at the column's rows")


if __name__ == "__main__":
    main()
