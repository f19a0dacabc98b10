#!/usr/bin/env python3
"""Closed-loop benchmark of the device MPC data path.

B vehicles run mpc_dynamics.main's receding-horizon loop (N = 30, dynamic bicycle,
incremental MPC) with every step on the GPU: reference search -> linearisation of
the N predicted stages -> QP assembly -> setup + solve -> plant step + shift
(osqp_amd.mpc_device.DynamicMPC).  Prints one JSON line: vehicle-steps/s on the
GPU and, beside it, the same step on the host (numpy restatement of the reference's
Python steps + the CPU oracle solve) for a bounded sample of vehicles.

  python tools/bench_loop.py --batch 8192 --steps 20 [--warm-start]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "python-mpc_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402


def initial_states(B, seed=5):
    rng = np.random.default_rng(seed)
    x0 = np.zeros((B, 6))
    x0[:, 1] = rng.uniform(-2, 2, B)
    x0[:, 2] = np.deg2rad(rng.uniform(-8, 8, B))
    x0[:, 3] = rng.uniform(10, 20, B)
    return x0, np.zeros((B, 2))


def host_steps(x0, u0, px, py, N, steps, seconds):
    """The reference's step on the host for a few vehicles (numpy linearisation and
    assembly, oracle solve, numpy shift); returns vehicle-steps/s (1 core)."""
    import pyoracle
    from osqp_amd import mpc
    from test_mpc_device import reference_search, shift
    veh = mpc.VehicleParams(dt=0.05)
    done, t0 = 0, time.perf_counter()
    for b in range(x0.shape[0]):
        xt = np.concatenate([x0[b], u0[b]])
        pred = [xt]
        xk = xt.copy()
        for i in range(N):
            Ad, Bd, gd = mpc.linearise_dynamics(veh, xk[None, :6], xk[None, 6:])
            xk = np.concatenate([Ad[0] @ xk[:6] + Bd[0] @ xk[6:] + gd[0], xk[6:]])
            pred.append(xk)
        pred = np.array(pred)
        for _ in range(steps):
            Xr = reference_search(px, py, pred.T[:6], 0.05, N)
            Ad, Bd, gd = mpc.linearise_dynamics(veh, pred[:N, :6], pred[:N, 6:])
            P, q, A, l, u = mpc.incremental_qp(list(Ad), list(Bd), list(gd), xt, Xr, mpc.DYN_Q, mpc.DYN_QN, mpc.DYN_R,
                                               N, mpc.DYN_XMIN_T, mpc.DYN_XMAX_T, mpc.DYN_DUMIN, -mpc.DYN_DUMIN)
            o = pyoracle.OSQP()
            o.setup(P, q, A, l, u, polish=False, warm_start=False)
            r = o.solve()
            xt, pred, _ = shift(r.x, Ad[0], Bd[0], gd[0], xt, veh, N)
            done += 1
        if time.perf_counter() - t0 > seconds:
            break
    return done / (time.perf_counter() - t0), done


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--N", type=int, default=30)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--warm-start", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    import torch
    from osqp_amd.mpc_device import DynamicMPC
    from test_mpc_device import path
    px, py = path()
    x0, u0 = initial_states(a.batch)
    ctl = DynamicMPC(x0, u0, px, py, N=a.N, warm_start=a.warm_start)
    for _ in range(a.warmup):
        ctl.step()
    torch.cuda.synchronize()
    iters = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        st, it = ctl.step()
        iters.append(it)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    it = torch.stack(iters).cpu().numpy()
    ok = float((st.cpu().numpy() == 1).mean())
    line = {"metric": "closed-loop vehicle-steps/s (device MPC loop, mpc_dynamics.main)",
            "value": a.batch * a.steps / dt, "unit": "vehicle-steps/s", "ms_per_step": dt / a.steps * 1e3,
            "config": {"vehicles": a.batch, "N": a.N, "n": ctl.layout.n, "m": ctl.layout.m,
                       "warm_start": a.warm_start, "steps": a.steps, "warmup": a.warmup,
                       "iters_mean": float(it.mean()), "iters_max_per_step_mean": float(it.max(axis=1).mean()),
                       "solved_frac_last": ok, "variant": ctl.solver.plan_info()["variant"]}}
    if not a.no_cpu:
        nv = 64
        rate, done = host_steps(x0[:nv], u0[:nv], px, py, a.N, 4, a.cpu_seconds)
        line["cpu_baseline"] = {"value": rate, "unit": "vehicle-steps/s", "cores": 1, "kind": "port",
                                "sample": f"{done} vehicle-steps (4 steps per vehicle) of the reference's Python step "
                                          "restated in numpy + oracle solve (osqp not installed)"}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
