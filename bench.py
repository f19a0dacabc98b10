#!/usr/bin/env python3
"""bench.py -- batched MPC QP solves/sec on MI355X (BASELINE.json metric).

Workload (default, BASELINE.json configs[1]): B = 1024 lane-tracking QPs per
GPU, horizon N = 20, nx = 4, nu = 1 (vanilla lateral MPC layout of
Control/MPC/mpc_kinematics.py:148-200 with the lateral model of
vehicle_lateral_mpc_slack_increment.py:32-43), fp64, synthetic initial states.
One step = one pass of the hot path over the batch: osqp setup() + solve() for
every instance (Ruiz scaling, KKT factorisation, ADMM to eps 1e-3, unscaling)
-- the reference's per-call pattern (mpc_kinematics.py:194-198), with the
inputs already resident in HBM when the timed region starts.  Every step solves
a DIFFERENT batch: the same vehicles with their initial states jittered by
+-2 % of the D2 ranges (a receding-horizon proxy: nearby problems, as in the
reference's closed loops), so the solver's longest-previous-solve-first
dispatch (kernels.hip::k_order) predicts each step from the previous, different
QP -- never from a repeat of the same one.

Multi-GPU: one process per GPU.  Under torch.distributed.run (WORLD_SIZE set)
each process is one rank; `python bench.py --gpus N` without it spawns the N
rank processes itself (bench.launch: fresh interpreters, 127.0.0.1 rendezvous,
the parent never touches a GPU) and exits with their status.  Every rank solves
its own shard (no data-path collective); timing = barrier + synchronize on both
sides, max over ranks.  --config 3/5 select the slack / incremental-dynamic
workloads (not the headline line); cfg 5 is warm-started as SURVEY.md §8d D2
prescribes (cold solve, one-stage shift, timed warm re-solve).  --config 4 is
BASELINE.json configs[3]: ONE batch of 262144 slack QPs split into contiguous
shards over the N ranks (262144 / N per rank, strong scaling).  The batch is
built from 64 seeded chunks of 4096 instances (seed 4000 + chunk), so the union
of the shards is the same 262144 instances at every N and each rank builds only
its own chunks.

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
# MPCQP_PKG: diagnostic A/B of another build of the package (tools/gpu_ab2.sh)
sys.path.insert(0, os.environ.get("MPCQP_PKG", os.path.join(ROOT, "python-mpc_amd")))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

JITTER = 0.02  # per-step jitter of the initial states, fraction of the D2 half-range
# D2 ranges of the initial-state rows [:nx0] of l = u, per layout; the
# jittered states are clipped to them (cfg 5's accel at its bound would make x~_0 infeasible)
X0_RANGES = {
    "vanilla": [(-.05, .05), (-.1, .1), (-10 * np.pi / 180, 10 * np.pi / 180), (-3., 3.)],
    "slack": [(-.05, .05), (-.1, .1), (-10 * np.pi / 180, 10 * np.pi / 180), (-3., 3.),
              (-5 * np.pi / 180, 5 * np.pi / 180)],
    "dynamic": [(0., 0.), (0., 0.), (-np.pi / 8, np.pi / 8), (5., 25.), (-.5, .5), (-.2, .2),
                (-5 * np.pi / 180, 5 * np.pi / 180), (-1., 1.)],
}
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
FP64_PEAK_TFLOPS = 78.6  # MI355X fp64 vector peak (spec) -- diagnostic only


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 4, 5])
    ap.add_argument("--batch", type=int, default=None,
                    help="instances per GPU (default: the config's; cfg 4: the GLOBAL batch, split over the ranks)")
    ap.add_argument("--jitter", type=float, default=JITTER,
                    help="per-step jitter of the initial states, fraction of the D2 half-range")
    ap.add_argument("--independent", action="store_true",
                    help="every step's initial states drawn afresh from the D2 ranges (no correlation between steps)")
    ap.add_argument("--assemble", action="store_true",
                    help="lateral layouts (cfg 2/3/4): each step builds q, l, u on the device from the instances' "
                         "(x0, xr, bound regime) (SURVEY.md §8f F1) and solves with one shared P, A -- timed "
                         "from x0 alone; a separate metric, not the headline")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--separate-setup", action="store_true",
                    help="setup() and solve() as two kernels (default: mpcqp_setup_solve_device, fused where possible)")
    ap.add_argument("--one-shot", action=argparse.BooleanOptionalAction, default=True,
                    help="mpcqp_set_one_shot (default on): the fused kernel keeps no workspace state for later "
                         "calls -- the reference's fresh OSQP() + setup() + solve() per call "
                         "(mpc_kinematics.py:194-198); outputs bit-identical to --no-one-shot's persisting kernel")
    ap.add_argument("--fuse-warm", action=argparse.BooleanOptionalAction, default=True,
                    help="cfg 5: setup() + warm_start() as one call (mpcqp_setup_warm_device, default on; one "
                         "kernel where the wide batch setup applies), identical results to the two calls")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="diagnostic: no HIP events in the timed region (roofline kernel_ms from the untimed pass)")
    ap.add_argument("--no-dispatch-ab", action="store_true",
                    help="skip the identity-dispatch diagnostic (rocprof passes: one handle's launches only)")
    ap.add_argument("--no-pcie", action="store_true",
                    help="skip the PCIe-inclusive diagnostic (host buffers in, host buffers out)")
    ap.add_argument("--no-latency", action="store_true",
                    help="skip the per-call latency diagnostic (one cfg-5 QP through the osqp shim)")
    return ap.parse_args(argv)


def dist_env():
    """(world, rank, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def instance_seed(config, rank):
    """Each rank solves its own shard of synthetic instances (weak scaling)."""
    return 1000 * config + rank


CHUNK = 4096  # cfg 4: instances per seeded chunk of the global batch


def make_shard(config, B, world, rank):
    """The rank's instances.  cfg 4 (strong scaling): contiguous chunks [r C / N, (r + 1) C / N)
    of the one global batch of B instances, chunk c generated with seed 4000 + c, so the
    shards of any world size tile the same global batch.  Other configs (weak scaling): B
    instances of the rank's own seed."""
    from osqp_amd import mpc
    if config != 4:
        return mpc.make_batch(config, B=B, seed=instance_seed(config, rank))
    if B % CHUNK or (B // CHUNK) % world:
        raise SystemExit(f"cfg 4: the global batch {B} must be a multiple of {CHUNK} * world ({world})")
    nc = B // CHUNK
    parts = [mpc.make_batch(4, B=CHUNK, seed=instance_seed(4, c))
             for c in range(rank * nc // world, (rank + 1) * nc // world)]
    b = dict(parts[0])
    for k in ("Px", "Ax", "q", "l", "u"):
        b[k] = np.ascontiguousarray(np.concatenate([p[k] for p in parts]))
    b["B"] = B // world
    return b


def launch(n, cmd, timeout=None, stdout=None):
    """Run `cmd` as n rank processes of one job (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*
    as torch.distributed.run sets them, rendezvous on 127.0.0.1).  Fresh interpreters are
    started as children; the caller must not have touched a GPU.  Returns the first
    non-zero exit status (the remaining ranks are stopped then), else 0."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=env, stdout=stdout))
    t0 = time.monotonic()
    rc = 0
    while procs:
        for p in list(procs):
            c = p.poll()
            if c is None:
                continue
            procs.remove(p)
            if c and not rc:
                rc = c
                for q in procs:
                    q.terminate()
        if timeout is not None and time.monotonic() - t0 > timeout and procs:
            rc = rc or 124
            for q in procs:
                q.kill()
        time.sleep(0.05)
    return rc


def cpu_share():
    """(cores this process may run on, where the count comes from): the affinity mask,
    capped by a cgroup v2 CPU quota when one is set (a GPU lease's share of the host)."""
    n = len(os.sched_getaffinity(0))
    src = f"sched_getaffinity ({n})"
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()
        if quota != "max":
            q = max(1, int(-(-int(quota) // int(period))))
            if q < n:
                n, src = q, f"cgroup cpu.max quota {quota}/{period} (affinity {src})"
    except (OSError, ValueError):
        pass
    return n, src


def max_over_ranks(x, world):
    """Max of a host float over all ranks (gloo; no data-path collective)."""
    if world <= 1:
        return float(x)
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(x)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def x0_sequence(b, count, seed, jitter=JITTER, independent=False):
    """`count` initial-state arrays (B, nx0) of batch `b`: the first its own, each later one
    jittered (`jitter` of the D2 half-range, clipped to the D2 ranges) or, `independent`,
    drawn afresh from the D2 ranges."""
    from osqp_amd import mpc
    rng = np.random.default_rng(seed + 7919)
    lo, hi = (np.array(v) for v in zip(*X0_RANGES[mpc.CONFIGS[b["cfg"]]["layout"]]))
    x0 = -b["l"][:, :lo.size]
    seq = [x0]
    for _ in range(count - 1):
        if independent:
            seq.append(lo + (hi - lo) * rng.uniform(0, 1, x0.shape))
        else:
            seq.append(np.clip(x0 + jitter * 0.5 * (hi - lo) * rng.uniform(-1, 1, x0.shape), lo, hi))
    return seq


def bound_sequence(b, count, seed, to_dev, jitter=JITTER, independent=False):
    """`count` distinct (l, u) device pairs of batch `b`: the initial-state rows (l = u = -x0)
    from x0_sequence; everything else of the QP (P, A, q, the other bounds) is shared."""
    xs = x0_sequence(b, count, seed, jitter, independent)
    nx0 = xs[0].shape[1]
    dl0, du0 = to_dev(b["l"]), to_dev(b["u"])
    seq = [(dl0, du0)]
    for xt in xs[1:]:
        dxt = to_dev(-xt)
        dl, du = dl0.clone(), du0.clone()
        dl[:, :nx0] = dxt
        du[:, :nx0] = dxt
        seq.append((dl, du))
    return seq


def theta_sequence(b, count, seed, to_dev, jitter=JITTER, independent=False):
    """The same steps as parameters theta = (x0, xr) of the lateral assembler (F1,
    osqp_amd.mpc_device.LateralAssembler): the device builds q, l, u from them."""
    xs = x0_sequence(b, count, seed, jitter, independent)
    out = []
    for xt in xs:
        th = b["theta"].copy()
        th[:, :xt.shape[1]] = xt
        out.append(to_dev(th))
    return out


def solve_kernel_name(info, fused):
    """The kernel the roofline times: the fused setup+solve kernel where the four- or
    two-wave variant runs it (solve_wave.hip::k_setup_solve_w4 / _w2), else the solve
    kernel."""
    v = info["variant"]
    if v in (10, 17) and fused:
        return "mpcqp::k_setup_solve_w4" if v == 17 else "mpcqp::k_setup_solve_w2"
    return {8: "mpcqp::k_solve_w", 9: "mpcqp::k_solve_w", 10: "mpcqp::k_solve_w2", 17: "mpcqp::k_solve_w4",
            11: "mpcqp::k_solve_b", 12: "mpcqp::k_solve_b", 13: "mpcqp::k_solve_b", 14: "mpcqp::k_solve_b",
            16: "mpcqp::k_solve_d"}.get(v, "mpcqp::k_solve")


def pmc_traffic(workload, batch, kernel, one_shot=False):
    """HBM bytes per k_solve launch from rocprofv3 PMC passes committed under
    profiles/ (tools/gpu_profile.sh + tools/pmc_summary.py give traffic.json, copied to profiles/traffic_<workload>_b<B>.json:
    FETCH_SIZE and WRITE_SIZE from separate --pmc passes, FETCH_SIZE doubled per
    the gfx950 note of MI355X_MICROARCH.md).  {} when not measured.  The record names the code it
    was measured on (code_sha16: tools/codeobj.py's hash of every instantiation of the kernel in the
    library); when that is not the loaded library's, the record is stale -- {"traffic_stale": True}.
    one_shot: the one-shot form's record (traffic_<workload>_b<B>_oneshot.json)."""
    path = os.path.join(ROOT, "profiles", f"traffic_{workload}_b{batch}{'_oneshot' if one_shot else ''}.json")
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        t = json.load(f)
    if t.get("kernel") != kernel:
        return {}  # measured on another kernel: not this one's traffic
    try:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import codeobj
        import osqp_amd
        cur = codeobj.kernel_code_hash(osqp_amd.LIB_PATH, kernel)
    except Exception as e:  # (tools absent: the record cannot be tied to this build)
        return {"traffic_stale": True, "stale_reason": f"code hash unavailable: {e}", "source": t.get("source")}
    if t.get("code_sha16") != cur:
        return {"traffic_stale": True, "code_sha16": cur, "source": t.get("source"),
                "stale_reason": f"measured on code {t.get('code_sha16')}, loaded {cur}"}
    return t


def copy_peak(dev_index, nbytes=2 << 30, reps=10):
    """Achievable HBM bandwidth of a device-to-device copy: libmpcqp's streaming copy kernel
    (mpcqp_debug_copy: 16-byte non-temporal loads and stores, four per lane in flight, the
    MI355X guide's float4-copy form, which measures ~6.3 TB/s) over a 2 GiB buffer `reps`
    times, (read + write) bytes / time, GB/s.  Outside the timed region."""
    import ctypes as C
    import torch
    import osqp_amd
    dev = torch.device("cuda", dev_index)
    src = torch.empty(nbytes // 8, dtype=torch.float64, device=dev).fill_(1.0)
    dst = torch.empty_like(src)
    torch.cuda.synchronize(dev)
    ms = C.c_double()
    stream = torch.cuda.current_stream(dev).cuda_stream
    rc = osqp_amd.lib().mpcqp_debug_copy(src.data_ptr(), dst.data_ptr(), src.numel(), reps, stream, C.byref(ms))
    if rc != 0:
        raise RuntimeError(osqp_amd.lib().mpcqp_last_error().decode())
    if not torch.equal(dst[:: 1 << 20], src[:: 1 << 20]):
        raise RuntimeError("copy_peak: the copy kernel's output differs from its input")
    gbs = 2 * nbytes / (ms.value * 1e-3) / 1e9
    del src, dst
    torch.cuda.empty_cache()
    return gbs


class PinnedHost:
    """Host buffers from hipHostMalloc for the PCIe leg (torch's pin_memory blocks made the
    uploads stall the host thread for milliseconds now and then on the box), and
    hipMemcpyAsync on a stream handle -- no torch copy bookkeeping between the calls."""

    def __init__(self):
        import ctypes
        self.C = ctypes
        self.hip = ctypes.CDLL("libamdhip64.so")
        self.hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                            ctypes.c_void_p]
        self.hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
        self.hip.hipHostFree.argtypes = [ctypes.c_void_p]
        self.owned = []

    def like(self, t):
        import torch
        C = self.C
        if isinstance(t, np.ndarray):
            t = torch.from_numpy(np.ascontiguousarray(t))
        nbytes = max(t.numel() * t.element_size(), 8)
        ptr = C.c_void_p()
        if self.hip.hipHostMalloc(C.byref(ptr), nbytes, 0) != 0:
            raise RuntimeError("hipHostMalloc failed")
        self.owned.append(ptr.value)
        h = torch.frombuffer((C.c_char * nbytes).from_address(ptr.value), dtype=t.dtype, count=t.numel())
        h = h.view(t.shape)
        h.copy_(t.cpu())
        return h

    def copy(self, dst, src, kind, stream):  # kind: 1 host to device, 2 device to host
        if self.hip.hipMemcpyAsync(dst.data_ptr(), src.data_ptr(), dst.numel() * dst.element_size(), kind,
                                   stream.cuda_stream) != 0:
            raise RuntimeError("hipMemcpyAsync failed")

    def free(self):
        for ptr in self.owned:
            self.hip.hipHostFree(ptr)
        self.owned = []


def pcie_leg(solver, dev, local, bufs, host_in, outs, pin, steps, mode, warmup=8, ctx=None):
    """PCIe-inclusive rate (diagnostic, never `value`): every step copies
    the batch's Px, Ax, q, l, u from pinned host memory (PinnedHost) to HBM, runs the same
    mpcqp_setup_solve_device call as the timed step, and copies x, y, status, iters back to
    pinned host memory.  mode:
      "serial":    all of it in order on one torch stream, passed to the library as the
                   caller stream;
      "pipelined": two sets of device buffers, the kernels on the handle's own stream, the
                   copies on a torch stream in the order H2D(i), D2H(i-1): step i's inputs go
                   up while step i-1's kernel runs, and i-1's outputs come down while step i's
                   kernel runs (the overlap a host-side caller of the batch API can get).
    (Measured, round 4: an upload whose stream waits for a kernel blocks the calling host
    thread until that kernel is done -- hipMemcpyAsync returned after 0.3-0.5 ms -- so the
    host cannot run ahead; the pipelined form still hides the uploads behind the previous
    kernel.  A variant with the downloads behind each kernel on its own stream measured no
    better, profiles/r4s2_pcie/.)  Python's cyclic collector is off inside the timed loop.
    bufs: [(dPx, dAx, dq, dl, du, dx, dy, dst, dit)] x (1 or 2); host_in: [(hPx, hAx, hq,
    hl, hu)] cycled over the steps; outs: two sets of host outputs.  ctx: a dict that keeps the
    copy stream and the events from pass to pass (round 5: a stream created per pass made the
    first pipelined pass of a run the slowest, 0.75-0.85 ms against 0.45-0.57).  Returns s per step."""
    import gc
    import torch
    H2D, D2H = 1, 2
    # the copy stream at high priority: HIP puts it on a hardware queue of its own, not on one
    # it may share (GPU_MAX_HW_QUEUES = 4) with the handle's stream -- a shared queue runs the
    # copies and kernels in one order and the pipelined leg fell to the serial rate in about
    # one pass of three (0.72 against 0.45 ms per step, round 4)
    ctx = {} if ctx is None else ctx
    if "cs" not in ctx:
        ctx["cs"] = torch.cuda.Stream(dev, priority=-1)
        ctx["ks"] = torch.cuda.ExternalStream(solver.stream_handle().value, device=torch.device("cuda", local))
        ctx["ready"] = [torch.cuda.Event() for _ in range(2)]
        ctx["done"] = [torch.cuda.Event() for _ in range(2)]
    cs, ks, ready, done = ctx["cs"], ctx["ks"], ctx["ready"], ctx["done"]
    piped = mode == "pipelined"

    def down(i):
        for hh, dd in zip(outs[i % 2], bufs[i % len(bufs)][5:]):
            pin.copy(hh, dd, D2H, cs)

    def run(i):
        k = i % len(bufs)
        d = bufs[k]
        for dd, hh in zip(d[:5], host_in[i % len(host_in)]):
            pin.copy(dd, hh, H2D, cs)
        if not piped:
            solver.setup_solve(*d[:5], *d[5:], stream=cs.cuda_stream)
            down(i)
            return
        ready[k].record(cs)
        if i > 0:
            cs.wait_event(done[(i - 1) % 2])
            down(i - 1)
        ks.wait_event(ready[k])
        solver.setup_solve(*d[:5], *d[5:])
        done[k].record(ks)

    def drain(i):
        if piped and i > 0:
            cs.wait_event(done[(i - 1) % 2])
            down(i - 1)

    solver.synchronize()
    for i in range(warmup):
        run(i)
    drain(warmup)
    torch.cuda.synchronize(dev)
    solver.synchronize()
    gc_on = gc.isenabled()
    gc.disable()
    try:
        t0 = time.perf_counter()
        for i in range(steps):
            run(i)
        drain(steps)
        torch.cuda.synchronize(dev)
        solver.synchronize()
        return (time.perf_counter() - t0) / steps
    finally:
        if gc_on:
            gc.enable()


LATENCY_WORKLOAD = {
    5: "incremental-dynamic-N50, ONE QP (n 508, m 916), fresh OSQP()+setup()+solve() per call, cold "
       "(mpc_dynamics.py:392-396)",
    2: "vanilla-lateral-N20, ONE QP (n 104, m 188), fresh OSQP()+setup()+solve() per call "
       "(mpc_kinematics.py:194-198)",
}


def latency_leg(cfg=5, reps=30, warmup=3):
    """Per-call latency of the reference's Control/MPC call pattern, never `value`: a fresh
    osqp.OSQP() + setup() + solve() of ONE QP every call (Control/MPC/mpc_dynamics.py:392-396,
    mpc_kinematics.py:194-198), through the `import osqp` shim on the GPU, beside the oracle
    (one host thread) doing the same calls on the same QP.  The QP: instance 0 of the cfg-5
    generator (incremental dynamic MPC, N = 50, cold start as mpc_increment sets it), or of the
    cfg-2 generator (the vanilla lateral layout of mpc_kinematics.mpc, N = 20).  Medians over
    `reps` calls; per-iteration figures divide the whole call by the ADMM iterations."""
    import pyoracle
    from osqp_amd import OSQP, mpc
    b = mpc.make_batch(cfg, B=1, seed=1)
    P, A = b["P"].copy(), b["A"].copy()
    P.data, A.data = b["Px"][0].copy(), b["Ax"][0].copy()
    q, l, u = b["q"][0].copy(), b["l"][0].copy(), b["u"][0].copy()
    settings = {k: v for k, v in b["settings"].items() if k != "verbose"}
    out = {}
    for name, cls in (("gpu", OSQP), ("cpu", pyoracle.OSQP)):
        ts, tv, it = [], [], 0
        for r in range(warmup + reps):
            t0 = time.perf_counter()
            o = cls()
            o.setup(P, q, A, l, u, **settings)
            t1 = time.perf_counter()
            res = o.solve()
            t2 = time.perf_counter()
            del o
            if r >= warmup:
                ts.append(t1 - t0)
                tv.append(t2 - t1)
                it = int(res.info.iter)
                st = res.info.status
        tot = float(np.median(np.add(ts, tv)))
        out[name] = {"call_ms": tot * 1e3, "setup_ms": float(np.median(ts)) * 1e3,
                     "solve_ms": float(np.median(tv)) * 1e3, "iters": it, "status": st,
                     "us_per_iter": tot * 1e6 / max(1, it), "solve_us_per_iter": float(np.median(tv)) * 1e6 / max(1, it)}
    out["cpu"]["threads"] = 1
    out.update(workload=LATENCY_WORKLOAD[cfg],
               reps=reps, gpu_over_cpu_call=out["gpu"]["call_ms"] / out["cpu"]["call_ms"],
               method="host arrays through the osqp shim (osqp_amd.OSQP) vs oracle/osqp_oracle.c (pyoracle.OSQP, one "
                      "thread); medians; us_per_iter = the whole call / ADMM iterations")
    return out


def main(argv=None, solver_cls=None, device=None):
    """argv: the command line (default sys.argv[1:]).  solver_cls / device: a stand-in for
    osqp_amd.DeviceBatch and its torch device -- only tests/test_multiproc.py passes them,
    to rehearse the rank logic on CPU (the stand-in is defined in tests/, never here)."""
    args = parse(argv)
    world, rank, local = dist_env()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # one process per GPU: spawn the ranks (this process stays off the GPU) and exit
        # with their status; rank 0 prints the JSON line
        cmd = [sys.executable, os.path.abspath(__file__)] + (sys.argv[1:] if argv is None else list(argv))
        raise SystemExit(launch(args.gpus, cmd))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} ranks were started")
    if os.environ.get("MPCQP_BENCH_SHARE_GPU") == "1":
        # diagnostic: every rank on GPU 0, to rehearse the N > 1 path (ranks, gloo barriers,
        # max over ranks, rank 0's line) on a one-GPU box; never for a measurement
        local = 0
    import torch
    import torch.distributed as dist
    from osqp_amd import DeviceBatch, _drop_common_zeros

    json_fd = 1
    if world > 1:
        # gloo prints its "[Gloo] Rank r is connected to ..." lines on stdout (from C++): send
        # the ranks' stdout to stderr and keep the original for rank 0's one JSON line
        sys.stdout.flush()
        json_fd = os.dup(1)
        os.dup2(2, 1)
        dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
    if device is None:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device(device)
    on_gpu = dev.type == "cuda"
    dsync = torch.cuda.synchronize if on_gpu else (lambda: None)
    Solver = solver_cls or DeviceBatch

    from osqp_amd import mpc
    spec = mpc.CONFIGS[args.config]
    strong = args.config == 4  # one global batch split over the ranks
    if strong:
        B_global = args.batch or spec["B"]
        B = B_global // world
    else:
        B = args.batch or spec["B"]
        B_global = world * B
    b = make_shard(args.config, B_global if strong else B, world, rank)
    P, Px = _drop_common_zeros(b["P"], b["Px"])
    A, Ax = _drop_common_zeros(b["A"], b["Ax"])
    settings = {k: v for k, v in b["settings"].items() if k != "verbose"}
    n, m = b["n"], b["m"]

    def to_dev(a, dtype=torch.float64):
        return torch.from_numpy(np.ascontiguousarray(a)).to(dev, dtype=dtype).contiguous()

    dPx, dAx, dq = (to_dev(a) for a in (Px, Ax, b["q"]))
    # the base batch, then one distinct batch per warmup and timed step
    nsteps = 1 + args.warmup + args.steps
    if args.assemble:
        if b.get("theta") is None:
            raise SystemExit("--assemble: the lateral layouts only (cfg 2, 3, 4)")
        from osqp_amd.mpc_device import LateralAssembler
        asm = LateralAssembler(spec["layout"], N=b["N"], device=local)
        dPx, dAx = (to_dev(v) for v in asm.matrices())  # ONE P and A for the batch (shared-matrix mode)
        ths = theta_sequence(b, nsteps, instance_seed(args.config, rank), to_dev, jitter=args.jitter,
                             independent=args.independent)
        dreg = to_dev(b["regime"], dtype=torch.int32)
        dq = torch.empty((B, b["n"]), dtype=torch.float64, device=dev)
        dlv = torch.empty((B, b["m"]), dtype=torch.float64, device=dev)
        duv = torch.empty((B, b["m"]), dtype=torch.float64, device=dev)
        seq = [(dlv, duv)] * nsteps
    else:
        seq = bound_sequence(b, nsteps, instance_seed(args.config, rank), to_dev,
                             jitter=args.jitter, independent=args.independent)
    dl, du = seq[0]
    dx = torch.empty((B, n), dtype=torch.float64, device=dev)
    dy = torch.empty((B, m), dtype=torch.float64, device=dev)
    dst = torch.empty(B, dtype=torch.int32, device=dev)
    dit = torch.empty(B, dtype=torch.int32, device=dev)
    dsync()
    solver = Solver(P, A, B, device=local, **settings)
    warm = args.config == 5
    one_shot = bool(args.one_shot and not warm and not args.separate_setup and hasattr(solver, "one_shot")
                    and solver.one_shot(True))
    xs = ys = None
    fuse_warm = bool(warm and args.fuse_warm and hasattr(solver, "setup_warm"))
    if warm:
        # SURVEY.md §8d D2, cfg 5 ("warm-started ADMM"): solve once cold, shift the solution
        # one stage as the reference shifts its horizon (mpc_dynamics.py:589-610), and time
        # setup + warm start from the shifted (x, y) + solve
        from osqp_amd.mpc_device import warm_shift
        solver.setup(dPx, dAx, dq, dl, du)
        solver.solve(dx, dy, dst, dit)
        solver.synchronize()
        xs, ys = warm_shift(b["N"], 8, 2, dx, dy)
        dsync()

    def step(t, sv=solver, fused=not args.separate_setup):
        sl, su = seq[t]
        if args.assemble:  # F1: q, l, u from theta on the device, on the solver's stream order
            asm.assemble(ths[t], dreg, out=(dq, sl, su), stream=sv.stream_handle())
        if warm and fuse_warm:  # setup + warm start in one call (mpcqp_setup_warm_device), then the solve
            sv.setup_warm(dPx, dAx, dq, sl, su, xs, ys)
            sv.solve(dx, dy, dst, dit)
        elif warm:  # setup, then the warm start, then the solve
            sv.setup(dPx, dAx, dq, sl, su)
            sv.warm_start(xs, ys)
            sv.solve(dx, dy, dst, dit)
        elif fused:  # mpcqp_setup_solve_device: one kernel where the solve kernel allows it
            sv.setup_solve(dPx, dAx, dq, sl, su, dx, dy, dst, dit)
        else:
            sv.setup(dPx, dAx, dq, sl, su)
            sv.solve(dx, dy, dst, dit)

    step(0)  # the base batch: its statuses / iterations are the ones the CPU baseline is compared with
    solver.synchronize()
    # (copies: on a CPU device .cpu() would alias the buffers the later steps overwrite)
    status = dst.cpu().numpy().copy()
    iters = dit.cpu().numpy().copy()
    # the base batch's control block, for the CPU baseline's parity figure (rank 0, N = 1)
    u_base = dx[:, b["u_block"]].cpu().numpy().copy() if (rank == 0 and world == 1 and not args.no_cpu) else None
    for t in range(1, 1 + args.warmup):
        step(t)
    solver.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    barrier()
    dsync()
    solver.synchronize()
    fused = not (warm or args.separate_setup)
    # Kernel time, live in the timed region.  A fused step is ONE kernel, and the steps run
    # back to back on the solver's stream, so one HIP event pair on that stream around the
    # K steps gives the average launch duration with nothing between the kernels (an event
    # pair per launch puts two event packets between consecutive kernels: ≈12 us per step).
    # Other steps (setup kernel + solve kernel, cfg 5's warm start) keep an event pair per
    # launch, which separates the solve kernel's time.
    span = None
    if not args.no_kernel_timing:
        # (a batch past kOrderFuseMax = 16384 runs the order sort as a second kernel per step)
        if fused and not args.assemble and B <= 16384 and on_gpu and hasattr(solver, "stream_handle"):
            ext = torch.cuda.ExternalStream(solver.stream_handle().value, device=torch.device("cuda", local))
            span = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True), ext)
        else:
            solver.timing(True, setup=not fused)
    t0 = time.perf_counter()
    if span:
        span[0].record(span[2])
    for t in range(1 + args.warmup, 1 + args.warmup + args.steps):
        step(t)
    if span:
        span[1].record(span[2])
    solver.synchronize()
    dsync()
    t1 = time.perf_counter()
    barrier()
    if span:
        kt = {"setup_ms": 0.0, "n_setup": 0, "solve_ms": span[0].elapsed_time(span[1]), "n_solve": args.steps,
              "method": "one HIP event pair on the solver's stream around the timed steps / steps"}
    else:
        kt = solver.timing_read() if not args.no_kernel_timing else None
        if kt:
            kt["method"] = "a HIP event pair around every solve launch in the timed region"
    iters_last = dit.cpu().numpy()  # the last timed step's batch (the flop model's iteration count)
    solver.timing(False)
    if args.no_kernel_timing:  # diagnostic: kernel times from a few untimed steps
        solver.timing(True, setup=not fused)
        for t in range(1 + args.warmup, 1 + args.warmup + min(5, args.steps)):
            step(t)
        solver.synchronize()
        kt = solver.timing_read()
        kt["method"] = "a HIP event pair around every solve launch, untimed steps"
        solver.timing(False)
    dt = max_over_ranks(t1 - t0, world)

    # Diagnostic A/B, outside the timed region and never `value`: the same sequence of
    # batches on a handle that dispatches in identity order (MPCQP_DISPATCH=identity)
    # instead of longest-previous-solve-first (kernels.hip::k_order).
    value_identity = None
    if not args.no_dispatch_ab:
        os.environ["MPCQP_DISPATCH"] = "identity"
        ident = Solver(P, A, B, device=local, **settings)
        del os.environ["MPCQP_DISPATCH"]
        if one_shot:
            ident.one_shot(True)
        for t in range(1 + args.warmup):
            step(t, ident)
        ident.synchronize()
        ta = time.perf_counter()
        for t in range(1 + args.warmup, 1 + args.warmup + args.steps):
            step(t, ident)
        ident.synchronize()
        value_identity = B * args.steps / (time.perf_counter() - ta)
        del ident

    # Diagnostic, outside the timed region and never `value`: the rate with the batch handed
    # over in host memory (the PCIe-inclusive line of DESIGN.md §6)
    pcie = None
    if (rank == 0 and world == 1 and on_gpu and not args.no_pcie and not args.assemble and not warm and fused
            and B <= 65536 and hasattr(solver, "stream_handle")):
        import torch as _t
        ph = PinnedHost()
        try:
            hPx, hAx, hq = ph.like(Px), ph.like(Ax), ph.like(b["q"])
            host_in = [(hPx, hAx, hq, ph.like(seq[t][0]), ph.like(seq[t][1]))
                       for t in range(1 + args.warmup, 1 + args.warmup + min(4, args.steps))]
            set0 = (dPx, dAx, dq, dl.clone(), du.clone(), dx, dy, dst, dit)
            set1 = tuple(t.clone() for t in set0)
            outs = [tuple(ph.like(t) for t in set0[5:]) for _ in range(2)]
            # five passes of each, alternated, on one copy stream (a warm-up pass of each first)
            ser, pip, ctx = [], [], {}
            pcie_leg(solver, dev, local, [set0], host_in, outs, ph, args.steps, "serial", ctx=ctx)
            pcie_leg(solver, dev, local, [set0, set1], host_in, outs, ph, args.steps, "pipelined", ctx=ctx)
            for _ in range(5):
                ser.append(pcie_leg(solver, dev, local, [set0], host_in, outs, ph, args.steps, "serial", ctx=ctx))
                pip.append(pcie_leg(solver, dev, local, [set0, set1], host_in, outs, ph, args.steps, "pipelined",
                                    ctx=ctx))
        finally:
            _t.cuda.synchronize(dev)
            solver.synchronize()
            ph.free()
        t_ser, t_pip = float(np.median(ser)), float(np.median(pip))
        h2d = 8 * (Px.shape[1] + Ax.shape[1] + n + 2 * m)
        d2h = 8 * (n + m) + 8
        pcie = {"value_serial": B / t_ser, "ms_per_step_serial": t_ser * 1e3,
                "value_pipelined": B / t_pip, "ms_per_step_pipelined": t_pip * 1e3,
                "passes_ms_serial": [round(v * 1e3, 4) for v in ser],
                "passes_ms_pipelined": [round(v * 1e3, 4) for v in pip],
                "h2d_bytes_per_solve": h2d, "d2h_bytes_per_solve": d2h,
                "method": "hipHostMalloc host buffers: H2D of Px, Ax, q, l, u, the same setup_solve call, D2H "
                          "of x, y, status, iters every step; serial on one stream / pipelined over two "
                          "buffer sets, copies on their own stream beside the kernels (bench.py::pcie_leg); "
                          "the median of five alternated passes of each after an untimed one, one copy stream "
                          "for all; never `value`",
                "spread_pipelined": (max(pip) - min(pip)) / float(np.median(pip)),
                "spread_serial": (max(ser) - min(ser)) / float(np.median(ser))}
        del set1

    value = B_global * args.steps / dt
    nnzP, nnzA = P.nnz, A.nnz
    # SURVEY.md §8d D3 counts the nonzeros of one instance's matrices: cfg 5's stored
    # pattern is the union over the batch (2666 entries), of which an instance has about
    # 2016 nonzero -- the algorithmic bytes count the instance's own (mean over the batch)
    nnzP_alg = float(np.count_nonzero(Px) / B)
    nnzA_alg = float(np.count_nonzero(Ax) / B)
    bytes_per_solve = 8 * (nnzP_alg + nnzA_alg + n + 2 * m) + 8 * (n + m) + (8 * (n + m) if warm else 0)
    if args.assemble:  # from the parameters: theta in, x and y out (P, A shared: read once per launch)
        bytes_per_solve = 8 * ths[0].shape[1] + 4 + 8 * (n + m)
    solve_ms = kt["solve_ms"] / max(1, kt["n_solve"])
    setup_ms = kt["setup_ms"] / kt["n_setup"] if kt["n_setup"] else None  # None: setup runs inside the fused kernel
    achieved = bytes_per_solve * B / (solve_ms * 1e-3) / 1e9
    info = solver.plan_info()
    # fp64 flop model per ADMM iteration (diagnostic): BT solve 3*nb*S^2 FMAs, A/A' products,
    # elementwise ~12 flops per row/column
    S = info["block"]
    flop_iter = 2 * (3 * info["nb"] * S * S + 2 * nnzA) + 12 * (n + m)
    fp64_tflops = flop_iter * float(iters_last.astype(np.float64).sum()) / (solve_ms * 1e-3) / 1e12

    traffic = pmc_traffic(spec["name"], B, solve_kernel_name(info, fused=fused), one_shot)
    copy_gbs = copy_peak(local) if (on_gpu and rank == 0 and not args.no_cpu) else None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        import pyoracle
        threads, threads_src = cpu_share()
        # bounded sample: passes over the same instances until ~cpu_seconds of wall time
        nc = min(B, max(threads * 8, 64))
        done, tc, passes, t_setup, t_solve = 0, 0.0, 0, 0.0, 0.0
        ws = {}
        if warm:
            ws = dict(x0=xs[:nc].cpu().numpy(), y0=ys[:nc].cpu().numpy())
        while tc < args.cpu_seconds and passes < 10000:
            t = time.perf_counter()
            rc = pyoracle.solve_batch(P, A, Px[:nc], b["q"][:nc], Ax[:nc], b["l"][:nc], b["u"][:nc],
                                      nthreads=threads, **ws, **settings)
            tc += time.perf_counter() - t
            t_setup += rc.t_setup
            t_solve += rc.t_solve
            done += nc
            passes += 1
        cpu = {"value": done / tc, "unit": "QP solves/s", "cores": threads, "kind": "port",
               "cores_source": threads_src, "host_cpus": os.cpu_count(),
               "sample": f"{passes} passes over the first {nc} of the {B} instances ({done} solves), "
                         f"fresh setup(){'+warm_start(shifted x, y)' if warm else ''}+solve() each, "
                         f"{threads} POSIX threads, oracle/osqp_oracle.c "
                         f"(OSQP 0.6 restatement; osqp itself is not installed on the box)",
               "seconds": round(tc, 3),
               # thread-seconds of the two phases (orc_setup: scaling, KKT ordering and
               # LDL' factorisation; orc_solve: ADMM) and the solve-only rate they imply
               "setup_thread_s": round(t_setup, 3), "solve_thread_s": round(t_solve, 3),
               "value_solve_only": done / tc * (t_setup + t_solve) / t_solve if t_solve > 0 else None,
               "status_match_gpu": float(np.mean(rc.status_val == status[:nc])),
               "iter_match_gpu": float(np.mean(rc.iter == iters[:nc])),
               # north-star tolerance ||u* - u*_ref||_inf < 1e-4: the largest difference over
               # the sampled instances' control blocks (GPU base-batch solve vs the oracle's)
               "parity_max_du": float(np.nanmax(np.abs(u_base[:nc] - rc.x[:, b["u_block"]])))}

    latency = None
    if rank == 0 and world == 1 and on_gpu and not args.no_cpu and not args.no_latency:
        latency = latency_leg(5)
        latency["cfg2"] = latency_leg(2)  # (the kinematic scripts' call, the headline layout)

    if rank == 0:
        kname = solve_kernel_name(info, fused=fused)
        line = {
            "metric": ("QP solves/sec (batch) at N=20 nx=4 nu=1" if args.config == 2 else
                       f"QP solves/sec (batch), {spec['name']}") +
                      (", incl. on-device QP assembly from x0 (F1, shared P/A)" if args.assemble else ""),
            "value": value,
            "unit": "QP solves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded lane-tracking initial states, SURVEY.md §8d D2, " +
                    ("drawn afresh every step)" if args.independent else f"jittered +-{args.jitter:.0%} per step)"),
            "config": {"workload": spec["name"], "config_index": args.config, "batch_per_gpu": B,
                       "global_batch": B_global, "horizon_N": b["N"], "n": n, "m": m,
                       "nnz_triuP": nnzP, "nnz_A": nnzA, "nnz_A_per_instance": nnzA_alg,
                       "eps_abs": 1e-3, "eps_rel": 1e-3,
                       "step": ("setup()+warm_start(base solution shifted one stage)+solve()" +
                                (" (mpcqp_setup_warm_device: setup + warm start one call"
                                 + (", one kernel)" if solver.setup_warm_fused() else ")") if fuse_warm else "")
                                if warm else
                                "setup()+solve()" + ("" if args.separate_setup else
                                                     f" (mpcqp_setup_solve_device: one call; kernel {kname}"
                                                     + (", one-shot: no workspace state kept)" if one_shot else ")")))
                               + " per instance, inputs resident in HBM; a distinct batch per step (" +
                               ("initial states drawn afresh)" if args.independent else
                                f"initial states jittered +-{args.jitter:.0%} of the D2 ranges)"),
                       "one_shot": one_shot,
                       "fuse_warm": fuse_warm,
                       "parallelism": f"batch-shard x{world}",
                       "dispatch": "longest previous solve first (kernels.hip::k_order), predicted from the "
                                   "previous step's different batch",
                       "value_identity_dispatch_rank0": value_identity,
                       "iters_mean": float(iters.mean()), "iters_max": int(iters.max()),
                       "solved_frac": float(np.mean(status == 1)),
                       "plan": {"nb": info["nb"], "block": S, "amax": info["amax"], "npad": info["npad"],
                                "lds_bytes": info["lds_bytes_solve"],
                                "kernel_variant": info["variant"], "threads_per_qp": info["threads_per_qp"]}},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic.get("bytes_per_launch"),
                         "traffic_stale": bool(traffic.get("traffic_stale", False)),
                         "traffic_code_sha16": traffic.get("code_sha16"),
                         # the achievable peak of a plain device copy on this
                         # GPU, beside the datasheet peak (diagnostic; `frac` uses the datasheet)
                         "peak_copy_measured": copy_gbs,
                         "frac_of_copy_peak": (achieved / copy_gbs) if copy_gbs else None,
                         "traffic_source": traffic.get("source"),
                         "kernel": kname,
                         "kernel_ms": solve_ms, "kernel_ms_method": kt.get("method"), "setup_kernel_ms": setup_ms,
                         "bytes_per_solve": bytes_per_solve, "launch_instances": B,
                         "fp64_tflops_model": fp64_tflops, "fp64_peak_tflops": FP64_PEAK_TFLOPS},
            "cpu_baseline": cpu,
            "pcie_inclusive": pcie,
            "latency": latency,
        }
        if json_fd == 1:
            print(json.dumps(line), flush=True)
        else:
            sys.stdout.flush()
            os.write(json_fd, (json.dumps(line) + "\n").encode())
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
