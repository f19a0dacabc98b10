"""World-size-2 gloo rehearsal of bench.py's multi-GPU logic on the CPU.

bench.py shards the batch across ranks with no data-path collective (SURVEY.md
§8e E1): each rank builds its own synthetic instances (distinct seeds; cfg 4: its
contiguous chunks of one global batch) and the only collective is the max over
ranks of the timed region.  Here CPU ranks run that logic -- bench.main itself,
started by bench.launch (the `python bench.py --gpus N` path) with the oracle
stand-in of tests/_fake_batch.py in place of the GPU kernel, whose parity the -m gpu
tests cover (tests/test_multigpu.py: the shard / gather code on the device).
"""
import json
import subprocess
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


def test_bench_main_two_ranks(tmp_path):
    """`bench.py --gpus 2`: bench.launch starts two ranks of bench.main (here on CPU with
    the oracle stand-in); rank 0 prints one JSON line with the whole-job rate."""
    import bench
    out = tmp_path / "line.json"
    with open(out, "w") as f:
        rc = bench.launch(2, [sys.executable, os.path.join(ROOT, "tests", "bench_rank_cpu.py"), "--gpus", "2",
                              "--config", "2", "--batch", "16", "--steps", "2", "--warmup", "1",
                              "--no-dispatch-ab"], stdout=f, timeout=240)
    assert rc == 0
    lines = [ln for ln in open(out).read().splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["config"]["global_batch"] == 32
    assert d["config"]["batch_per_gpu"] == 16 and d["steps"] == 2
    assert abs(d["value"] - 32 * 2 / (d["ms_per_step"] * 2 / 1e3)) < 1e-6 * d["value"]
    assert d["cpu_baseline"] is None  # N = 1 only
    assert d["config"]["solved_frac"] == 1.0


def test_bench_rank_failure_stops_the_job(tmp_path):
    """A rank that fails ends the job with its status (the other rank is stopped)."""
    import bench
    code = "import os, sys, time; r = int(os.environ['RANK']); time.sleep(30 if r else 0); sys.exit(3 if r == 0 else 0)"
    t0 = __import__("time").monotonic()
    assert bench.launch(2, [sys.executable, "-c", code], timeout=60) == 3
    assert __import__("time").monotonic() - t0 < 20


def test_bench_gpus_must_match_world(monkeypatch):
    import bench
    monkeypatch.setenv("WORLD_SIZE", "1")
    with pytest.raises(SystemExit, match="WORLD_SIZE=1"):
        bench.main(["--gpus", "2"])


def test_cfg4_shards_tile_one_global_batch(monkeypatch):
    """cfg 4 (BASELINE configs[3], strong scaling): the shards of every world size are
    contiguous slices of the same global batch."""
    import bench
    monkeypatch.setattr(bench, "CHUNK", 8)
    full = bench.make_shard(4, 64, 1, 0)
    for world in (2, 4, 8):
        parts = [bench.make_shard(4, 64, world, r) for r in range(world)]
        assert all(p["B"] == 64 // world for p in parts)
        for k in ("Px", "Ax", "q", "l", "u"):
            assert np.array_equal(np.concatenate([p[k] for p in parts]), full[k])
    with pytest.raises(SystemExit):
        bench.make_shard(4, 60, 2, 0)


def test_bench_main_one_rank_cpu_baseline(tmp_path):
    """`bench.py` at N = 1 on CPU with the oracle stand-in: the cpu_baseline object -- the
    oracle timed on a bounded sample, its statuses / iterations / control blocks against the
    base-batch solve (parity_max_du; exactly 0 here, the stand-in being the oracle)."""
    out = tmp_path / "line.json"
    with open(out, "w") as f:
        rc = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "bench_rank_cpu.py"), "--config", "2",
                             "--batch", "16", "--steps", "2", "--warmup", "1", "--no-dispatch-ab",
                             "--cpu-seconds", "0.2"], stdout=f, timeout=240,
                            env=dict(os.environ, OMP_NUM_THREADS="2")).returncode
    assert rc == 0
    d = json.loads([ln for ln in open(out).read().splitlines() if ln.startswith("{")][-1])
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["value"] > 0 and cb["cores"] >= 1
    assert cb["status_match_gpu"] == 1.0 and cb["iter_match_gpu"] == 1.0
    assert cb["parity_max_du"] == 0.0
