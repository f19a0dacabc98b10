#!/usr/bin/env python3
"""bench.py -- batched MPC QP solves/sec on MI355X (BASELINE.json metric).

Workload (default, BASELINE.json configs[1]): B = 1024 lane-tracking QPs per
GPU, horizon N = 20, nx = 4, nu = 1 (vanilla lateral MPC layout of
Control/MPC/mpc_kinematics.py:148-200 with the lateral model of
vehicle_lateral_mpc_slack_increment.py:32-43), fp64, synthetic initial states.
One step = one pass of the hot path over the batch: osqp setup() + solve() for
every instance (Ruiz scaling, KKT factorisation, ADMM to eps 1e-3, unscaling)
-- the reference's per-call pattern (mpc_kinematics.py:194-198), with the
inputs already resident in HBM when the timed region starts.

Multi-GPU: one process per GPU (torch.distributed.run); every rank solves its
own batch (weak scaling, no data-path collective); timing = barrier +
synchronize on both sides, max over ranks.  --config 3/5 select the slack /
incremental-dynamic workloads (not the headline line); cfg 5 is warm-started as
SURVEY.md §8d D2 prescribes (cold solve, one-stage shift, timed warm re-solve).

rank 0 prints ONE JSON line with "roofline" (k_solve, HBM-bound by the
algorithmic-bytes model of SURVEY.md §8d D3, HIP-event kernel times from the
timed region) and "cpu_baseline" (the oracle -- CPU restatement of OSQP 0.6 --
timed on this host on a bounded sample of the same instances, N=1 only).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "python-mpc_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
FP64_PEAK_TFLOPS = 78.6  # MI355X fp64 vector peak (spec) -- diagnostic only


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 5])
    ap.add_argument("--batch", type=int, default=None, help="instances per GPU (default: the config's)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-dispatch-ab", action="store_true",
                    help="skip the identity-dispatch diagnostic (rocprof passes: one handle's launches only)")
    return ap.parse_args()


def dist_env():
    """(world, rank, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def instance_seed(config, rank):
    """Each rank solves its own shard of synthetic instances (weak scaling)."""
    return 1000 * config + rank


def max_over_ranks(x, world):
    """Max of a host float over all ranks (gloo; no data-path collective)."""
    if world <= 1:
        return float(x)
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(x)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def pmc_traffic(workload, batch):
    """HBM bytes per k_solve launch from rocprofv3 PMC passes committed under
    profiles/ (tools/pmc_traffic.py writes profiles/traffic_<workload>_b<B>.json:
    FETCH_SIZE and WRITE_SIZE from separate --pmc passes, FETCH_SIZE doubled per
    the gfx950 note of MI355X_MICROARCH.md).  {} when not measured."""
    path = os.path.join(ROOT, "profiles", f"traffic_{workload}_b{batch}.json")
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        return json.load(f)


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    from osqp_amd import DeviceBatch, mpc, _drop_common_zeros

    world, rank, local = dist_env()
    if world > 1:
        dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    spec = mpc.CONFIGS[args.config]
    B = args.batch or (spec["B"] if args.config != 4 else spec["B"] // 8)
    b = mpc.make_batch(args.config, B=B, seed=instance_seed(args.config, rank))
    P, Px = _drop_common_zeros(b["P"], b["Px"])
    A, Ax = _drop_common_zeros(b["A"], b["Ax"])
    settings = {k: v for k, v in b["settings"].items() if k != "verbose"}
    n, m = b["n"], b["m"]

    def to_dev(a, dtype=torch.float64):
        return torch.from_numpy(np.ascontiguousarray(a)).to(dev, dtype=dtype).contiguous()

    dPx, dAx, dq, dl, du = (to_dev(a) for a in (Px, Ax, b["q"], b["l"], b["u"]))
    dx = torch.empty((B, n), dtype=torch.float64, device=dev)
    dy = torch.empty((B, m), dtype=torch.float64, device=dev)
    dst = torch.empty(B, dtype=torch.int32, device=dev)
    dit = torch.empty(B, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    solver = DeviceBatch(P, A, B, device=local, **settings)
    warm = args.config == 5
    xs = ys = None
    if warm:
        # SURVEY.md §8d D2, cfg 5 ("warm-started ADMM"): solve once cold, shift the solution
        # one stage as the reference shifts its horizon (mpc_dynamics.py:589-610), and time
        # setup + warm start from the shifted (x, y) + solve
        from osqp_amd.mpc_device import warm_shift
        solver.setup(dPx, dAx, dq, dl, du)
        solver.solve(dx, dy, dst, dit)
        solver.synchronize()
        xs, ys = warm_shift(b["N"], 8, 2, dx, dy)
        torch.cuda.synchronize()

    def step(sv=solver):
        sv.setup(dPx, dAx, dq, dl, du)
        if warm:
            sv.warm_start(xs, ys)
        sv.solve(dx, dy, dst, dit)

    for _ in range(args.warmup):
        step()
    solver.synchronize()
    status = dst.cpu().numpy()
    iters = dit.cpu().numpy()

    def barrier():
        if world > 1:
            dist.barrier()

    barrier()
    torch.cuda.synchronize()
    solver.synchronize()
    solver.timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    solver.synchronize()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    kt = solver.timing_read()
    solver.timing(False)
    dt = max_over_ranks(t1 - t0, world)

    # Diagnostic A/B, outside the timed region and never `value`: the same steps on a
    # handle that dispatches in identity order (MPCQP_DISPATCH=identity) instead of
    # longest-previous-solve-first (kernels.hip::k_order).  The bench re-solves one
    # batch, so there the previous iteration counts predict the next ones exactly.
    value_identity = None
    if not args.no_dispatch_ab:
        os.environ["MPCQP_DISPATCH"] = "identity"
        ident = DeviceBatch(P, A, B, device=local, **settings)
        del os.environ["MPCQP_DISPATCH"]
        step(ident)
        ident.synchronize()
        ta = time.perf_counter()
        for _ in range(args.steps):
            step(ident)
        ident.synchronize()
        value_identity = B * args.steps / (time.perf_counter() - ta)
        del ident

    value = world * B * args.steps / dt
    nnzP, nnzA = P.nnz, A.nnz
    bytes_per_solve = 8 * (nnzP + nnzA + n + 2 * m) + 8 * (n + m) + (8 * (n + m) if warm else 0)
    solve_ms = kt["solve_ms"] / max(1, kt["n_solve"])
    setup_ms = kt["setup_ms"] / max(1, kt["n_setup"])
    achieved = bytes_per_solve * B / (solve_ms * 1e-3) / 1e9
    info = solver.plan_info()
    # fp64 flop model per ADMM iteration (diagnostic): BT solve 3*nb*S^2 FMAs, A/A' products,
    # elementwise ~12 flops per row/column
    S = info["block"]
    flop_iter = 2 * (3 * info["nb"] * S * S + 2 * nnzA) + 12 * (n + m)
    fp64_tflops = flop_iter * float(iters.astype(np.float64).sum()) / (solve_ms * 1e-3) / 1e12

    traffic = pmc_traffic(spec["name"], B)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        import pyoracle
        threads = int(os.environ.get("OMP_NUM_THREADS") or min(16, os.cpu_count() or 1))
        # bounded sample: passes over the same instances until ~cpu_seconds of wall time
        nc = min(B, max(threads * 8, 64))
        done, tc, passes = 0, 0.0, 0
        ws = {}
        if warm:
            ws = dict(x0=xs[:nc].cpu().numpy(), y0=ys[:nc].cpu().numpy())
        while tc < args.cpu_seconds and passes < 10000:
            t = time.perf_counter()
            rc = pyoracle.solve_batch(P, A, Px[:nc], b["q"][:nc], Ax[:nc], b["l"][:nc], b["u"][:nc],
                                      nthreads=threads, **ws, **settings)
            tc += time.perf_counter() - t
            done += nc
            passes += 1
        cpu = {"value": done / tc, "unit": "QP solves/s", "cores": threads, "kind": "port",
               "sample": f"{passes} passes over the first {nc} of the {B} instances ({done} solves), "
                         f"fresh setup(){'+warm_start(shifted x, y)' if warm else ''}+solve() each, "
                         f"{threads} POSIX threads, oracle/osqp_oracle.c "
                         f"(OSQP 0.6 restatement; osqp itself is not installed on the box)",
               "seconds": round(tc, 3),
               "status_match_gpu": float(np.mean(rc.status_val == status[:nc])),
               "iter_match_gpu": float(np.mean(rc.iter == iters[:nc]))}

    if rank == 0:
        line = {
            "metric": "QP solves/sec (batch) at N=20 nx=4 nu=1" if args.config == 2 else
                      f"QP solves/sec (batch), {spec['name']}",
            "value": value,
            "unit": "QP solves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded lane-tracking initial states, SURVEY.md §8d D2)",
            "config": {"workload": spec["name"], "config_index": args.config, "batch_per_gpu": B,
                       "global_batch": world * B, "horizon_N": b["N"], "n": n, "m": m,
                       "nnz_triuP": nnzP, "nnz_A": nnzA, "eps_abs": 1e-3, "eps_rel": 1e-3,
                       "step": ("setup()+warm_start(previous solution shifted one stage)+solve()" if warm else
                                "setup()+solve()") + " per instance, inputs resident in HBM",
                       "parallelism": f"batch-shard x{world}",
                       "dispatch": "longest previous solve first (kernels.hip::k_order)",
                       "value_identity_dispatch_rank0": value_identity,
                       "iters_mean": float(iters.mean()), "iters_max": int(iters.max()),
                       "solved_frac": float(np.mean(status == 1)),
                       "plan": {"nb": info["nb"], "block": S, "amax": info["amax"], "lds_bytes": info["lds_bytes_solve"],
                                "kernel_variant": info["variant"], "threads_per_qp": info["threads_per_qp"]}},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic.get("bytes_per_launch"),
                         "traffic_source": traffic.get("source"),
                         "kernel": {64: "mpcqp::k_solve_w", 128: "mpcqp::k_solve_w2"}.get(info["threads_per_qp"], "mpcqp::k_solve"),
                         "kernel_ms": solve_ms, "setup_kernel_ms": setup_ms,
                         "bytes_per_solve": bytes_per_solve, "launch_instances": B,
                         "fp64_tflops_model": fp64_tflops, "fp64_peak_tflops": FP64_PEAK_TFLOPS},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
