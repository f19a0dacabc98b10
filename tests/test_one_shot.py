"""One-shot fused setup + solve (mpcqp_set_one_shot).

The reference's Control/MPC call pattern builds a fresh osqp.OSQP(), calls setup() and solve()
and drops the object (mpc_kinematics.py:194-198), so nothing reads the workspace afterwards.
The one-shot form of the fused four-wave kernel keeps the scaled problem and the G blocks on chip
and stores no warm-start iterates or certificates (solve_wave.hip, setup_r.h ONE).  These
tests hold it to the persisting kernel bit for bit -- x, y, status, iteration count -- on the
cfg-2 headline batch and a cfg-3 sample, over two calls (the second one runs in the LPT dispatch
order the first call's iteration counts set), and check that the calls which read the workspace
refuse to run after a one-shot call until a setup.
"""
import numpy as np
import pytest

from osqp_amd import mpc


def _inputs(cfg, B, seed, dev):
    import torch
    from osqp_amd import _drop_common_zeros
    b = mpc.make_batch(cfg, B=B, seed=seed)
    P, Px = _drop_common_zeros(b["P"], b["Px"])
    A, Ax = _drop_common_zeros(b["A"], b["Ax"])
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    s = {k: v for k, v in b["settings"].items() if k != "verbose"}
    rng = np.random.default_rng(seed + 1)
    # a second call's bounds: the first call's, moved (a new measured state per instance)
    l2, u2 = b["l"].copy(), b["u"].copy()
    fin = np.isfinite(l2) & np.isfinite(u2) & (l2 == u2)
    shift = rng.normal(scale=0.05, size=l2.shape)
    l2[fin] += shift[fin]
    u2[fin] += shift[fin]
    return P, A, s, (t(Px), t(Ax), t(b["q"])), [(t(b["l"]), t(b["u"])), (t(l2), t(u2))], b


def _out(B, n, m, dev):
    import torch
    return (torch.empty((B, n), dtype=torch.float64, device=dev), torch.empty((B, m), dtype=torch.float64, device=dev),
            torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.int32, device=dev))


def _same_bits(a, c):
    """Bit-identical (NaN outputs of unsolved instances included); on a mismatch, which
    instances differ and their status / iterations."""
    import torch
    ab, cb = (t.view(torch.int64) if t.dtype == torch.float64 else t for t in (a, c))
    if torch.equal(ab, cb):
        return True
    rows = (ab != cb).reshape(ab.shape[0], -1).any(1).nonzero().flatten().tolist()
    raise AssertionError(f"{len(rows)} instances differ, first {rows[:8]}; max |diff| "
                         f"{(a - c).abs().nan_to_num(0).max().item() if a.dtype == torch.float64 else None}")


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,B", [(2, 1024), (3, 4096)])
def test_one_shot_is_bit_identical(cfg, B):
    import torch
    from osqp_amd import DeviceBatch
    dev = torch.device("cuda", 0)
    P, A, s, (Px, Ax, q), bounds, b = _inputs(cfg, B, 31, dev)
    torch.cuda.synchronize()  # (the handles' streams are not ordered with torch's)
    keep, one = DeviceBatch(P, A, B, device=0, **s), DeviceBatch(P, A, B, device=0, **s)
    # cfg 2: the G blocks in an LDS region of their own; cfg 3 (two workgroups per CU leave no
    # room for one): straight into the solve's copy (factorize_w4_gl)
    assert one.one_shot(True) == {2: 2, 3: 3}[cfg]
    for call, (l, u) in enumerate(bounds):
        o1, o2 = _out(B, b["n"], b["m"], dev), _out(B, b["n"], b["m"], dev)
        keep.setup_solve(Px, Ax, q, l, u, *o1)
        one.setup_solve(Px, Ax, q, l, u, *o2)
        torch.cuda.synchronize()
        st = o1[2].cpu().numpy()
        for a, c in zip(o1, o2):
            assert _same_bits(a, c), np.unique(st, return_counts=True)
        if call == 0:  # (the moved bounds of the second call leave some instances infeasible)
            assert (o1[2] == 1).float().mean().item() > 0.99
    # the workspace is gone: the calls that read it refuse, until a setup
    o = _out(B, b["n"], b["m"], dev)
    with pytest.raises(ValueError, match="one-shot"):
        one.solve(*o)
    with pytest.raises(ValueError, match="one-shot"):
        one.update(q=q)
    with pytest.raises(ValueError, match="one-shot"):
        one.warm_start(x=o[0])
    one.setup(Px, Ax, q, *bounds[1])
    one.solve(*o)
    keep.setup(Px, Ax, q, *bounds[1])
    o1 = _out(B, b["n"], b["m"], dev)
    keep.solve(*o1)
    torch.cuda.synchronize()
    for a, c in zip(o1, o):
        assert _same_bits(a, c)


@pytest.mark.gpu
def test_one_shot_elsewhere_runs_as_usual():
    """cfg 5 (the long-horizon kernel): the one-shot switch does not apply; setup_solve runs the
    persisting path and the workspace stays usable (a warm start + solve after it)."""
    import torch
    from osqp_amd import DeviceBatch
    dev = torch.device("cuda", 0)
    B = 256
    P, A, s, (Px, Ax, q), bounds, b = _inputs(5, B, 7, dev)
    torch.cuda.synchronize()
    h = DeviceBatch(P, A, B, device=0, **s)
    assert h.one_shot(True) == 0
    o = _out(B, b["n"], b["m"], dev)
    h.setup_solve(Px, Ax, q, *bounds[0], *o)
    h.warm_start(o[0], o[1])
    o2 = _out(B, b["n"], b["m"], dev)
    h.solve(*o2)
    torch.cuda.synchronize()
    assert (o2[2] == 1).all()
