"""World-size-2 gloo rehearsal of bench.py's multi-GPU logic on the CPU.

bench.py shards the batch across ranks with no data-path collective (SURVEY.md
§8e E1): each rank builds its own synthetic instances (distinct seeds) and the
only collective is the max over ranks of the timed region.  Here two CPU ranks
run that logic, and each solves a few of its instances with the oracle (the GPU
kernel needs a device; its parity is covered by the -m gpu tests).
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "python-mpc_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch.distributed as dist
    import bench
    import pyoracle
    from osqp_amd import mpc
    w, r, _ = bench.dist_env()
    dist.init_process_group("gloo", init_method="env://", rank=r, world_size=w)
    b = mpc.make_batch(2, B=4, seed=bench.instance_seed(2, r))
    res = pyoracle.solve_batch(b["P"], b["A"], b["Px"], b["q"], b["Ax"], b["l"], b["u"], nthreads=1,
                               **{k: v for k, v in b["settings"].items() if k != "verbose"})
    tmax = bench.max_over_ranks(1.0 + r, w)
    np.savez(os.path.join(out, f"rank{r}.npz"), l=b["l"], status=res.status_val, tmax=tmax)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharding(tmp_path):
    import torch.multiprocessing as tmp
    world = 2
    tmp.spawn(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r0 = np.load(tmp_path / "rank0.npz")
    r1 = np.load(tmp_path / "rank1.npz")
    assert float(r0["tmax"]) == float(r1["tmax"]) == 2.0        # max over ranks
    assert not np.allclose(r0["l"], r1["l"])                    # distinct shards (x0 differs)
    assert np.all(r0["status"] == 1) and np.all(r1["status"] == 1)
