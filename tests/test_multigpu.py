"""The multi-device shard / gather path of the C ABI on the GPU.

mpcqp_setup_batch splits the batch into contiguous shards, one stream and workspace
per shard, enqueues every shard's kernels before gathering the results into the
caller's buffers (api.hip).  On the one-GPU box MPCQP_SPLIT=k cuts k shards on the
same device, so the b0 offsets and the launch-all-then-gather code run for real and
must give the unsharded results bit for bit.  BASELINE.json configs[3] (262144 slack
QPs over 8 GPUs) is exercised at one rank's full shard: 32768 instances.
"""
import numpy as np
import pytest

from parity import check_agreement
import pyoracle
from osqp_amd import OSQPBatch, mpc

pytestmark = pytest.mark.gpu


def _solve(b, monkeypatch, split, **s):
    if split > 1:
        monkeypatch.setenv("MPCQP_SPLIT", str(split))
    else:
        monkeypatch.delenv("MPCQP_SPLIT", raising=False)
    h = OSQPBatch()
    h.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
    assert h.plan_info()["n_devices"] == split
    r1 = h.solve()
    # a second solve after update(l, u): the shards' dispatch orders are their own
    l, u = b["l"].copy(), b["u"].copy()
    l[:, :2] *= 0.9
    u[:, :2] *= 0.9
    h.update(l=l, u=u)
    r2 = h.solve()
    # a matrix update (mpcqp_update_matrices_batch: each shard's slice of the values)
    h.update(Px=b["Px"] * 1.25, Ax=b["Ax"][:, ::2] * 0.95, Ax_idx=np.arange(0, b["Ax"].shape[1], 2))
    r3 = h.solve()
    return r1, r2, r3


@pytest.mark.parametrize("cfg,B,split", [(2, 1000, 3), (3, 257, 2), (5, 40, 4)])
def test_split_shards_are_bit_identical(monkeypatch, cfg, B, split):
    b = mpc.make_batch(cfg, B=B, seed=61)
    s = {k: v for k, v in b["settings"].items() if k != "verbose"}
    ref = _solve(b, monkeypatch, 1, **s)
    got = _solve(b, monkeypatch, split, **s)
    for rr, rg in zip(ref, got):
        for k in ("x", "y", "status_val", "iter", "obj_val", "pri_res", "dua_res", "prim_inf_cert", "dual_inf_cert"):
            assert np.array_equal(getattr(rr, k), getattr(rg, k), equal_nan=True), k


def test_cfg4_rank_shard_32768(monkeypatch):
    """One rank's shard of configs[3] (262144 / 8 = 32768 slack QPs, bench.make_shard):
    statuses and iteration counts against the oracle on a sample, and the second solve --
    dispatched longest-previous-first from the first solve's counts -- bit-identical to a
    handle that dispatches it in identity order."""
    import torch
    import bench
    from osqp_amd import DeviceBatch, _drop_common_zeros
    b = bench.make_shard(4, 262144, 8, 5)
    B = b["B"]
    assert B == 32768
    P, Px = _drop_common_zeros(b["P"], b["Px"])
    A, Ax = _drop_common_zeros(b["A"], b["Ax"])
    s = {k: v for k, v in b["settings"].items() if k != "verbose"}
    dev = torch.device("cuda", 0)

    def put(*arrs):
        return [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in arrs]

    def out():
        return (torch.empty((B, b["n"]), dtype=torch.float64, device=dev),
                torch.empty((B, b["m"]), dtype=torch.float64, device=dev),
                torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.int32, device=dev))

    l2 = b["l"].copy(); u2 = b["u"].copy()
    rng = np.random.default_rng(3)
    x0 = -l2[:, :5] + rng.uniform(-0.01, 0.01, (B, 5))
    l2[:, :5] = -x0; u2[:, :5] = -x0
    X = put(Px, Ax, b["q"], b["l"], b["u"])
    Y = put(Px, Ax, b["q"], l2, u2)
    lpt = DeviceBatch(P, A, B, device=0, **s)
    o1, o2 = out(), out()
    lpt.setup_solve(*X, *o1)
    lpt.setup_solve(*Y, *o2)
    lpt.synchronize()
    monkeypatch.setenv("MPCQP_DISPATCH", "identity")
    ref = DeviceBatch(P, A, B, device=0, **s)
    r2 = out()
    ref.setup_solve(*Y, *r2)
    ref.synchronize()
    for a, c in zip(o2, r2):
        assert torch.equal(a, c)
    st, it = o1[2].cpu().numpy(), o1[3].cpu().numpy()
    assert (st == 1).all()
    idx = np.random.default_rng(0).choice(B, 384, replace=False)
    bo = pyoracle.solve_batch(P, A, Px[idx], b["q"][idx], Ax[idx], b["l"][idx], b["u"][idx], nthreads=16, **s)
    bs = dict(b, P=P, A=A, Px=Px[idx], Ax=Ax[idx], q=b["q"][idx], l=b["l"][idx], u=b["u"][idx])
    check_agreement("cfg4 rank shard 32768, oracle sample 384", bs, o1[0].cpu().numpy()[idx],
                    o1[1].cpu().numpy()[idx], st[idx], it[idx], bo)
