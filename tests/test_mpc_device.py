"""Device MPC data path (csrc/mpc_device.hip) against host
restatements of the reference's steps and the reference's own fixtures.

  F2  linearise        vs tests/golden/linearise.npz (Vehicle_Dynamics.get_dynamics_model)
  F1  incr assembly    vs tests/golden/dyn_incr_n50.npz (mpc_increment's P, q, A, l, u)
  F3  reference search vs the restatement below of mpc_dynamics.py:30-90
      closed loop      each step decomposed: device Xr / Ad / QP / solution / shifted
                       horizon vs the host restatement of mpc_dynamics.main (:506-617)
                       fed the device's own state, with the solve checked against the
                       CPU oracle on the host-built QP.

The reference's own outputs pin those restatements (tests/golden/make_golden.py):
  refsearch.npz      reference_search / nearest_point (mpc_dynamics.py:30-90) on main()'s path
  dyn_main_n30.npz   three steps of mpc_dynamics.main (:437-617): each step's inputs, QP,
                     solution (the oracle's, behind the osqp stub) and shifted state
The host restatements are checked against them on CPU; the device kernels on the GPU.
The pattern test runs on CPU (layout creation is host-only); the rest needs the GPU.
"""
import json

import numpy as np
import pytest

from osqp_amd import canonical_data, mpc
from osqp_amd.mpc_device import DYN_MASK_A, DYN_MASK_B, IncrementalLayout

INF = 1e30  # OSQP_INFTY: bounds are clipped to it (osqp 0.6 osqp_setup / update_bounds)


def dense(M):
    return np.asarray(M.todense())


def _layout(N, **kw):
    return IncrementalLayout(N, mpc.DYN_Q, mpc.DYN_QN, mpc.DYN_R, mpc.DYN_XMIN_T, mpc.DYN_XMAX_T, mpc.DYN_DUMIN,
                             -mpc.DYN_DUMIN, **kw)


@pytest.mark.parametrize("N", [2, 3, 30, 50])
def test_layout_pattern_matches_host_builder(N):
    """The C layout's CSC templates equal mpc_increment's matrices (host builder, same
    structural nonzeros) after the osqp-python canonicalisation."""
    L = _layout(N)
    P, A, lt, ut = L.pattern()
    assert (L.n, L.m) == ((N + 1) * 8 + N * 2, (N + 1) * 8 + (N + 1) * 8 + N * 2)
    P2, _, A2, l2, u2 = mpc.incremental_qp([np.where(DYN_MASK_A, 7.0, 0.0)] * N, [np.where(DYN_MASK_B, 7.0, 0.0)] * N,
                                           [np.zeros(6)] * N, np.zeros(8), np.zeros((6, N + 1)), mpc.DYN_Q,
                                           mpc.DYN_QN, mpc.DYN_R, N, mpc.DYN_XMIN_T, mpc.DYN_XMAX_T, mpc.DYN_DUMIN,
                                           -mpc.DYN_DUMIN)
    P2, A2 = canonical_data(P2, A2)
    assert np.array_equal(P.indptr, P2.indptr) and np.array_equal(P.indices, P2.indices)
    assert np.array_equal(P.data, P2.data)
    assert np.array_equal(A.indptr, A2.indptr) and np.array_equal(A.indices, A2.indices)
    const = A2.data != 7.0
    assert np.array_equal(A.data[const], A2.data[const]) and not A.data[~const].any()
    ineq = slice((N + 1) * 8, None)
    assert np.array_equal(lt[ineq], np.clip(l2[ineq], -INF, INF))
    assert np.array_equal(ut[ineq], np.clip(u2[ineq], -INF, INF))


def test_layout_rejects_bad_arguments():
    for N in (0, 1):
        with pytest.raises(Exception):
            _layout(N)
    with pytest.raises(Exception):
        IncrementalLayout(10, mpc.DYN_Q, mpc.DYN_QN, mpc.DYN_R, mpc.DYN_XMIN_T, mpc.DYN_XMAX_T, mpc.DYN_DUMIN,
                          mpc.DYN_DUMIN - 1.0)  # dumin > dumax


# ------------------------------------------------------------------ host restatements --
def nearest_point(path_x, path_y, x, y, look_ind=0):
    """mpc_dynamics.py:30-41 (reversed scan, strict <)."""
    min_d, min_ind = np.inf, -1
    for i in reversed(range(len(path_x))):
        d = np.sqrt((path_x[i] - x) ** 2 + (path_y[i] - y) ** 2)
        if d < min_d:
            min_d, min_ind = d, i
    return min_ind + look_ind


def reference_search(path_x, path_y, pred_state, dt, N):
    """mpc_dynamics.py:44-90: pred_state (6, N+1) -> Xr (6, N+1)."""
    x_ref = np.zeros((6, N + 1))
    cumul_d = 0.0
    ind = nearest_point(path_x, path_y, pred_state[0, 0], pred_state[1, 0], look_ind=1)
    path_d = np.sqrt((path_x[ind + 1] - path_x[ind]) ** 2 + (path_y[ind + 1] - path_y[ind]) ** 2)
    for i in range(N + 1):
        cumul_d = cumul_d + abs(pred_state[3, i]) * dt
        while cumul_d >= path_d:
            ind = ind + 1
            path_d = path_d + np.sqrt((path_x[ind + 1] - path_x[ind]) ** 2 + (path_y[ind + 1] - path_y[ind]) ** 2)
        x_ref[0, i], x_ref[1, i], x_ref[3, i] = path_x[ind], path_y[ind], 10.0
    return x_ref


def path():
    """mpc_dynamics.main's path (:468-469): 200 points on y = 0.5 x + 5."""
    px = np.linspace(-10, 100, 200)
    return px, px * 0.5 + 5


def shift(sol, Ad0, Bd0, gd0, xt, veh, N):
    """Plant step + horizon shift of mpc_dynamics.main (:578-617) with the solution
    unpacked as in mpc_increment (:405-432).  The terminal Euler step
    (update_dynamics_model) is x + dt f(x, u), written here as Ad x + Bd u + gd of the
    linearisation at the same point (equal up to rounding)."""
    nx, nu, nxa = 6, 2, 8
    S = sol[:(N + 1) * nxa].reshape(N + 1, nxa)          # pred_x~ (stage-major)
    D = sol[(N + 1) * nxa:].reshape(N, nu)                # del_u
    u = xt[nx:] + D[0]
    x = Ad0 @ xt[:nx] + Bd0 @ u + gd0
    xt_new = np.concatenate([x, u])
    pred = np.empty((N + 1, nxa)); pdu = np.empty((N + 1, nu))
    pred[0] = xt_new
    pred[1:N] = S[2:N + 1]
    pdu[0:N - 1] = D[1:N]
    pdu[N - 1] = D[N - 1]
    Ae, Be, ge = mpc.linearise_dynamics(veh, S[N, :nx][None], S[N - 1, nx:][None])
    pred[N, :nx] = Ae[0] @ S[N, :nx] + Be[0] @ S[N - 1, nx:] + ge[0]
    pred[N, nx:] = pred[N - 1, nx:]
    pdu[N] = pdu[N - 1]
    return xt_new, pred, pdu


# ------------------------------------------- the restatements against the reference --
def test_reference_search_restatement_matches_reference(golden):
    """The host restatement above equals the reference's reference_search (captured:
    refsearch.npz, 64 predicted horizons on main()'s path, a quarter reversing)."""
    g = golden("refsearch.npz")
    N = g["pred"].shape[2] - 1
    for b in range(g["pred"].shape[0]):
        assert np.array_equal(reference_search(g["path_x"], g["path_y"], g["pred"][b], float(g["dt"]), N), g["Xr"][b])


def _main_qp(g, t):
    A = __import__("scipy.sparse", fromlist=["csc_matrix"]).csc_matrix(
        (g[f"A{t}_data"], g[f"A{t}_indices"], g[f"A{t}_indptr"]), shape=tuple(g[f"A{t}_shape"]))
    return g["P"], g["q"][t], A, g["l"][t], g["u"][t]


def test_main_steps_restatements_match_reference(golden):
    """Three steps of mpc_dynamics.main as the reference ran them (dyn_main_n30.npz): the
    host restatements -- linearisation, mpc_increment's QP, the plant step and horizon
    shift -- reproduce each step from the captured inputs and solution."""
    g = golden("dyn_main_n30.npz")
    veh = mpc.VehicleParams(dt=0.05)
    N = 30
    for t in range(g["in_xt"].shape[0]):
        pred = g["in_pred"][t].T                                  # (N+1, 8)
        Xr = reference_search(g["path_x"], g["path_y"], pred.T[:6], 0.05, N)
        assert np.array_equal(Xr, g["in_Xr"][t])
        Ad, Bd, gd = mpc.linearise_dynamics(veh, pred[:N, :6], pred[:N, 6:])
        assert np.allclose(Ad, g["in_Ad"][t], rtol=1e-13, atol=1e-15)
        assert np.allclose(Bd, g["in_Bd"][t], rtol=1e-13, atol=1e-15)
        assert np.allclose(gd, g["in_gd"][t], rtol=1e-12, atol=1e-13)
        P, q, A, l, u = mpc.incremental_qp(list(g["in_Ad"][t]), list(g["in_Bd"][t]), list(g["in_gd"][t]),
                                           g["in_xt"][t], g["in_Xr"][t], mpc.DYN_Q, mpc.DYN_QN, mpc.DYN_R, N,
                                           mpc.DYN_XMIN_T, mpc.DYN_XMAX_T, mpc.DYN_DUMIN, -mpc.DYN_DUMIN)
        Pr, qr, Ar, lr, ur = _main_qp(g, t)
        assert np.array_equal(dense(P), dense(Pr)) and np.array_equal(dense(A), dense(Ar))
        assert np.array_equal(q, qr) and np.array_equal(l, lr) and np.array_equal(u, ur)
        xt_new, pred_new, pdu_new = shift(g["sol"][t], g["in_Ad"][t][0], g["in_Bd"][t][0], g["in_gd"][t][0],
                                          g["in_xt"][t], veh, N)
        assert np.allclose(xt_new, g["out_xt"][t], rtol=1e-14, atol=1e-14)
        assert np.allclose(pred_new, g["out_pred"][t].T, rtol=1e-12, atol=1e-12)
        assert np.array_equal(pdu_new, g["out_pdu"][t].T)
    # consecutive steps chain: a step's output is the next step's input
    assert np.array_equal(g["out_xt"][:-1], g["in_xt"][1:]) and np.array_equal(g["out_pred"][:-1], g["in_pred"][1:])


# ------------------------------------------------------------------------- GPU tests --
@pytest.mark.gpu
def test_reference_search_matches_reference_fixture(golden):
    import torch
    from osqp_amd.mpc_device import reference_search as dev_search
    g = golden("refsearch.npz")
    pred = np.zeros((g["pred"].shape[0], g["pred"].shape[2], 8))
    pred[:, :, :6] = g["pred"].transpose(0, 2, 1)
    Xr = dev_search(torch.tensor(g["path_x"], device="cuda"), torch.tensor(g["path_y"], device="cuda"),
                    torch.tensor(pred, device="cuda"), float(g["dt"])).cpu().numpy()
    assert np.array_equal(Xr, g["Xr"])


@pytest.mark.gpu
def test_main_steps_on_device_match_reference(golden):
    """Each captured step of mpc_dynamics.main through the device kernels: reference search
    (bit-exact), linearisation, mpc_increment's QP, and the plant step + shift applied to
    the step's captured solution -- against the reference's own values; and the device
    solve of the step's QP against that solution."""
    import ctypes as C
    import torch
    import pyoracle
    from osqp_amd import OSQP
    from osqp_amd.mpc_device import Vehicle, _bind, _p, linearise, reference_search as dev_search
    g = golden("dyn_main_n30.npz")
    N, dev = 30, torch.device("cuda", 0)
    T = g["in_xt"].shape[0]
    L = _layout(N)
    veh = Vehicle(dt=0.05)
    t_ = lambda a: torch.tensor(np.ascontiguousarray(a), dtype=torch.float64, device=dev)
    pred = t_(g["in_pred"].transpose(0, 2, 1))                   # (T, N+1, 8)
    Xr = dev_search(t_(g["path_x"]), t_(g["path_y"]), pred, 0.05)
    assert np.array_equal(Xr.cpu().numpy(), g["in_Xr"])
    Ad, Bd, gd = linearise(veh, pred[:, :N, :6], pred[:, :N, 6:])
    assert np.allclose(Ad.cpu().numpy(), g["in_Ad"], rtol=1e-13, atol=1e-15)
    assert np.allclose(gd.cpu().numpy(), g["in_gd"], rtol=1e-12, atol=1e-13)
    Ax, q, l, u = L.assemble(t_(g["in_Ad"]), t_(g["in_Bd"]), t_(g["in_gd"]), t_(g["in_xt"]), t_(g["in_Xr"]))
    Apat = L.pattern()[1]
    for t in range(T):
        Pr, qr, Ar, lr, ur = _main_qp(g, t)
        A_dev = Apat.copy(); A_dev.data = Ax[t].cpu().numpy()
        assert np.allclose(dense(A_dev), dense(Ar), rtol=1e-15, atol=0)
        assert np.allclose(q[t].cpu().numpy(), qr, rtol=1e-15, atol=0)
        assert np.array_equal(l[t].cpu().numpy(), np.clip(lr, -INF, INF))
    # plant step + shift of the captured solutions
    xt = t_(g["in_xt"]); pr = pred.clone(); pdu = t_(g["in_pdu"].transpose(0, 2, 1))
    Lb = _bind()
    _check = __import__("osqp_amd", fromlist=["_check"])._check
    keep = [t_(g[k]) for k in ("sol", "in_Ad", "in_Bd", "in_gd")]  # alive until the kernel has run
    _check(Lb.mpcqp_incr_shift_device(L._h, C.byref(veh), T, *(_p(v) for v in keep), _p(xt), _p(pr), _p(pdu), None),
           "incr_shift")
    torch.cuda.synchronize()
    assert np.allclose(xt.cpu().numpy(), g["out_xt"], rtol=1e-14, atol=1e-14)
    assert np.allclose(pr.cpu().numpy(), g["out_pred"].transpose(0, 2, 1), rtol=1e-12, atol=1e-12)
    assert np.array_equal(pdu.cpu().numpy(), g["out_pdu"].transpose(0, 2, 1))
    # the solve of each captured QP: device and oracle agree, and the oracle reproduces the
    # solution the reference's loop ran on
    s = json.loads(str(g["settings"]))
    s.pop("verbose", None)
    for t in range(T):
        P, q_, A, l_, u_ = _main_qp(g, t)
        o = pyoracle.OSQP(); o.setup(P, q_, A, l_, u_, **s); ro = o.solve()
        assert np.array_equal(ro.x, g["sol"][t]) and ro.info.iter == g["sol_iter"][t]
        d = OSQP(); d.setup(P, q_, A, l_, u_, **s); rd = d.solve()
        assert rd.info.status == ro.info.status and rd.info.iter == ro.info.iter
        assert np.abs(rd.x[(N + 1) * 8:] - ro.x[(N + 1) * 8:]).max() < 1e-4

@pytest.mark.gpu
def test_linearise_matches_reference_fixture(golden):
    import torch
    from osqp_amd.mpc_device import Vehicle, linearise
    g = golden("linearise.npz")
    x = torch.tensor(g["x"], device="cuda"); u = torch.tensor(g["u"], device="cuda")
    x0, u0 = x.clone(), u.clone()
    Ad, Bd, gd = linearise(Vehicle(dt=float(g["dt"])), x, u)
    assert torch.equal(x, x0) and torch.equal(u, u0)  # the guard acts on copies
    assert np.allclose(Ad.cpu().numpy(), g["Ad"], rtol=1e-13, atol=1e-15)
    assert np.allclose(Bd.cpu().numpy(), g["Bd"], rtol=1e-13, atol=1e-15)
    assert np.allclose(gd.cpu().numpy(), g["gd"], rtol=1e-12, atol=1e-13)
    # horizon-shaped input with a strided view: (B, N, 6) taken from (B, N, 8)
    xt = torch.cat([x, u], dim=1).reshape(6, 8, 8)
    Ad3, Bd3, gd3 = linearise(Vehicle(dt=float(g["dt"])), xt[..., :6], xt[..., 6:])
    assert torch.equal(Ad3.reshape(48, 6, 6), Ad) and torch.equal(gd3.reshape(48, 6), gd)


@pytest.mark.gpu
def test_incremental_assembly_matches_reference_fixture(golden):
    import torch
    g = golden("dyn_incr_n50.npz")
    L = IncrementalLayout(50, g["Q"], g["QN"], g["R"], g["xmin_t"], g["xmax_t"], g["del_umin"], g["del_umax"])
    P, A, _, _ = L.pattern()
    T = g["q"].shape[0]
    dev = lambda a: torch.tensor(np.ascontiguousarray(a), dtype=torch.float64, device="cuda")
    Ax, q, l, u = L.assemble(dev(g["Ad"]), dev(g["Bd"]), dev(g["gd"][..., 0]), dev(g["xt0"]), dev(g["Xr"]))
    Ax, q, l, u = (t.cpu().numpy() for t in (Ax, q, l, u))
    for t in range(T):
        Pr = g["P"].copy(); Pr.data = g["Px"][t]
        Ar = g["A"].copy(); Ar.data = g["Ax"][t]
        A.data = Ax[t]
        assert np.array_equal(dense(P), dense(Pr))
        assert np.allclose(dense(A), dense(Ar), rtol=1e-15, atol=0)
        assert np.allclose(q[t], g["q"][t], rtol=1e-15, atol=0)
        assert np.array_equal(l[t], np.clip(g["l"][t], -INF, INF))
        assert np.array_equal(u[t], np.clip(g["u"][t], -INF, INF))


@pytest.mark.gpu
def test_reference_search_matches_restatement():
    import torch
    from osqp_amd.mpc_device import reference_search as dev_search
    px, py = path()
    rng = np.random.default_rng(3)
    B, N, dt = 64, 30, 0.05
    pred = np.zeros((B, N + 1, 8))
    s0 = rng.uniform(-5, 60, B)
    pred[:, :, 0] = s0[:, None] + rng.normal(0, 1, (B, 1))
    pred[:, :, 1] = 0.5 * s0[:, None] + 5 + rng.normal(0, 3, (B, 1))
    pred[:, :, 3] = rng.uniform(0, 30, (B, N + 1))
    pred[:B // 4, :, 3] *= -1  # reversing: |vx| is used
    Xr = dev_search(torch.tensor(px, device="cuda"), torch.tensor(py, device="cuda"),
                    torch.tensor(pred, device="cuda"), dt).cpu().numpy()
    for b in range(B):
        assert np.array_equal(Xr[b], reference_search(px, py, pred[b].T[:6], dt, N)), b


@pytest.mark.gpu
def test_reference_search_clamps_at_path_end():
    """Where the reference raises IndexError (its index reaches the last path point), the
    kernel holds the start of the last segment."""
    import torch
    from osqp_amd.mpc_device import reference_search as dev_search
    px, py = path()
    pred = np.zeros((1, 11, 8)); pred[0, :, 0] = 99.0; pred[0, :, 1] = 54.5; pred[0, :, 3] = 40.0
    Xr = dev_search(torch.tensor(px, device="cuda"), torch.tensor(py, device="cuda"),
                    torch.tensor(pred, device="cuda"), 0.05).cpu().numpy()
    assert np.all(Xr[0, 0] == px[-2]) and np.all(Xr[0, 1] == py[-2])


@pytest.mark.gpu
def test_closed_loop_matches_host_restatement():
    import pyoracle
    import torch
    from osqp_amd.mpc_device import DynamicMPC
    B, N, steps = 4, 30, 6
    x0 = np.zeros((B, 6)); x0[:, 3] = 15.0
    x0[:, 1] = [0.0, 1.0, -1.5, 0.5]; x0[:, 2] = np.deg2rad([0.0, 5.0, -3.0, 10.0])
    u0 = np.zeros((B, 2))
    px, py = path()
    ctl = DynamicMPC(x0, u0, px, py, N=N)
    veh = mpc.VehicleParams(dt=0.05)
    # initial guess (:513-522)
    xk = np.concatenate([x0, u0], 1)
    pred0 = [xk]
    for i in range(N):
        Ad, Bd, gd = mpc.linearise_dynamics(veh, xk[:, :6], xk[:, 6:])
        xk = np.concatenate([np.einsum("bij,bj->bi", Ad, xk[:, :6]) + np.einsum("bij,bj->bi", Bd, xk[:, 6:]) + gd,
                             xk[:, 6:]], 1)
        pred0.append(xk)
    assert np.allclose(ctl.pred.cpu().numpy(), np.stack(pred0, 1), rtol=1e-12, atol=1e-12)
    Apat = ctl.layout.pattern()[1]
    n_iter_match = 0
    for step in range(steps):
        xt, pred = ctl.xt.cpu().numpy(), ctl.pred.cpu().numpy()
        status, iters = ctl.step()
        status, iters = status.cpu().numpy(), iters.cpu().numpy()
        last = {k: v.cpu().numpy() for k, v in ctl.last.items()}
        sol = ctl.sol.cpu().numpy()
        for b in range(B):
            Xr = reference_search(px, py, pred[b].T[:6], 0.05, N)
            assert np.array_equal(last["Xr"][b], Xr)
            Ad, Bd, gd = mpc.linearise_dynamics(veh, pred[b, :N, :6], pred[b, :N, 6:])
            assert np.allclose(last["Ad"][b], Ad, rtol=1e-13, atol=1e-15)
            assert np.allclose(last["gd"][b], gd, rtol=1e-12, atol=1e-13)
            P, q, A, l, u = mpc.incremental_qp(list(Ad), list(Bd), list(gd), xt[b], Xr, mpc.DYN_Q, mpc.DYN_QN,
                                               mpc.DYN_R, N, mpc.DYN_XMIN_T, mpc.DYN_XMAX_T, mpc.DYN_DUMIN,
                                               -mpc.DYN_DUMIN)
            A_dev = Apat.copy(); A_dev.data = last["Ax"][b]
            assert np.allclose(dense(A_dev), dense(A), rtol=1e-12, atol=1e-15)
            assert np.allclose(last["q"][b], q, rtol=1e-12, atol=1e-12)
            assert np.allclose(last["l"][b], np.clip(l, -INF, INF), rtol=1e-12, atol=1e-14)
            o = pyoracle.OSQP()
            o.setup(P, q, A, l, u, polish=False, warm_start=False)
            ro = o.solve()
            assert status[b] == 1 and ro.info.status == "solved"
            n_iter_match += int(iters[b] == ro.info.iter)
            scale = max(1.0, np.abs(ro.x).max())
            assert np.abs(sol[b] - ro.x).max() < 1e-5 * scale, (step, b)
            du = slice((N + 1) * 8, None)
            assert np.abs(sol[b, du] - ro.x[du]).max() < 1e-4
            # plant step + shift from the device's own solution
            xt_new, pred_new, pdu_new = shift(sol[b], last["Ad"][b, 0], last["Bd"][b, 0], last["gd"][b, 0], xt[b],
                                              veh, N)
            assert np.allclose(ctl.xt[b].cpu().numpy(), xt_new, rtol=1e-13, atol=1e-13)
            assert np.allclose(ctl.pred[b].cpu().numpy(), pred_new, rtol=1e-10, atol=1e-10)
            assert np.allclose(ctl.pdu[b].cpu().numpy(), pdu_new, rtol=0, atol=0)
    assert n_iter_match >= 0.9 * B * steps
    # the vehicles converge toward the path (lateral error shrinks)
    xt = ctl.xt.cpu().numpy()
    assert np.all(np.isfinite(xt))


@pytest.mark.gpu
def test_warm_shift_moves_every_block_one_stage():
    import torch
    from osqp_amd.mpc_device import warm_shift
    N, nxa, nu, B = 7, 8, 2, 5
    n, m = (N + 1) * nxa + N * nu, 2 * (N + 1) * nxa + N * nu
    rng = np.random.default_rng(0)
    x = rng.standard_normal((B, n)); y = rng.standard_normal((B, m))
    xs, ys = warm_shift(N, nxa, nu, torch.tensor(x, device="cuda"), torch.tensor(y, device="cuda"))

    def shift(v, groups):
        out = []
        for g in range(groups):
            blk = v[:, g * (N + 1) * nxa:(g + 1) * (N + 1) * nxa].reshape(B, N + 1, nxa)
            out.append(np.concatenate([blk[:, 1:], blk[:, -1:]], 1).reshape(B, -1))
        du = v[:, groups * (N + 1) * nxa:].reshape(B, N, nu)
        out.append(np.concatenate([du[:, 1:], du[:, -1:]], 1).reshape(B, -1))
        return np.concatenate(out, 1)

    assert np.array_equal(xs.cpu().numpy(), shift(x, 1))
    assert np.array_equal(ys.cpu().numpy(), shift(y, 2))


@pytest.mark.gpu
def test_closed_loop_warm_start_matches_oracle():
    """warm_start=True (an extension): every step's solve starts from the previous
    solution shifted one stage; the oracle, warm-started from the same shifted iterates
    on the step's QP, gives the same controls.  Fewer iterations than the cold loop."""
    import pyoracle
    from osqp_amd.mpc_device import DynamicMPC
    B, N, steps = 64, 30, 6
    rng = np.random.default_rng(11)
    x0 = np.zeros((B, 6)); x0[:, 3] = rng.uniform(10, 20, B); x0[:, 1] = rng.uniform(-2, 2, B)
    x0[:, 2] = np.deg2rad(rng.uniform(-8, 8, B))
    px, py = path()
    cold = DynamicMPC(x0, np.zeros((B, 2)), px, py, N=N)
    warm = DynamicMPC(x0, np.zeros((B, 2)), px, py, N=N, warm_start=True)
    P, A, _, _ = warm.layout.pattern()
    Px = np.tile(P.data, (B, 1))
    du = slice((N + 1) * 8, None)
    ic = iw = match = 0
    prev = None
    for step in range(steps):
        sc, itc = cold.step()
        sw, itw = warm.step()
        ic += int(itc.sum()); iw += int(itw.sum())
        assert (sc.cpu().numpy() == 1).all() and (sw.cpu().numpy() == 1).all()
        last = {k: v.cpu().numpy() for k, v in warm.last.items()}
        ws = {} if prev is None else dict(x0=_stage_shift(prev[0], N, 8, 2, 1), y0=_stage_shift(prev[1], N, 8, 2, 2))
        ro = pyoracle.solve_batch(P, A, Px, last["q"], last["Ax"], last["l"], last["u"], nthreads=16, polish=False,
                                  **ws)
        x = warm.sol.cpu().numpy()
        same = ro.iter == itw.cpu().numpy()
        match += int(same.sum())
        assert np.abs(x[same][:, du] - ro.x[same][:, du]).max() < 1e-4
        prev = (x, warm.y.cpu().numpy())
    assert match >= 0.9 * B * steps
    assert iw < ic


def _stage_shift(v, N, nxa, nu, groups):
    B = v.shape[0]
    out = []
    for g in range(groups):
        blk = v[:, g * (N + 1) * nxa:(g + 1) * (N + 1) * nxa].reshape(B, N + 1, nxa)
        out.append(np.concatenate([blk[:, 1:], blk[:, -1:]], 1).reshape(B, -1))
    d = v[:, groups * (N + 1) * nxa:].reshape(B, N, nu)
    out.append(np.concatenate([d[:, 1:], d[:, -1:]], 1).reshape(B, -1))
    return np.concatenate(out, 1)


@pytest.mark.gpu
@pytest.mark.parametrize("layout,cfg,B", [("vanilla", 2, 1000), ("slack", 3, 777)])
def test_lateral_assembly_on_device(layout, cfg, B):
    """F1 for the lateral layouts (mpcqp_affine_apply_device): q, l, u of a seeded batch from
    its parameters (x0, xr) and bound regimes equal the host builders' bit for bit; the
    solve of the device-assembled batch with ONE shared P and A (mpcqp_set_shared_matrices)
    equals the solve of the host-built per-instance arrays bit for bit."""
    import torch
    from osqp_amd import DeviceBatch, _drop_common_zeros
    from osqp_amd.mpc_device import LateralAssembler
    b = mpc.make_batch(cfg, B=B, seed=21)
    rng = np.random.default_rng(5)
    theta = b["theta"].copy()
    theta[:, b["theta"].shape[1] - 4:] = rng.normal(size=(B, 4)) * 0.1   # a nonzero reference too
    dev = torch.device("cuda", 0)
    asm = LateralAssembler(layout, N=20, device=0)
    dth = torch.from_numpy(np.ascontiguousarray(theta)).to(dev)
    dreg = torch.from_numpy(b["regime"]).to(dev)
    q, l, u = asm.assemble(dth, dreg)
    torch.cuda.synchronize()
    qh, lh, uh = asm.map.evaluate(theta, b["regime"])
    for d, h in ((q, qh), (l, lh), (u, uh)):
        assert torch.equal(d.cpu(), torch.from_numpy(np.ascontiguousarray(h)))
    # the builder itself, instance by instance (a few)
    build = __import__("osqp_amd.mpc_device", fromlist=["lateral_builder"]).lateral_builder(layout, 20)[0]
    for k in (0, B // 2, B - 1):
        qr, lr, ur = build(theta[k], int(b["regime"][k]))
        assert np.array_equal(q[k].cpu().numpy(), qr) and np.array_equal(l[k].cpu().numpy(), lr)
    # solve: shared matrices + device vectors vs per-instance host arrays
    P, Px = _drop_common_zeros(b["P"], b["Px"])
    A, Ax = _drop_common_zeros(b["A"], b["Ax"])
    assert np.array_equal(Px[0], asm.matrices()[0]) and np.array_equal(Ax[0], asm.matrices()[1])
    s = {k: v for k, v in b["settings"].items() if k != "verbose"}

    def out():
        return (torch.empty((B, b["n"]), dtype=torch.float64, device=dev),
                torch.empty((B, b["m"]), dtype=torch.float64, device=dev),
                torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.int32, device=dev))

    h1, h2 = DeviceBatch(P, A, B, device=0, **s), DeviceBatch(P, A, B, device=0, **s)
    Pxs, Axs = (torch.from_numpy(np.ascontiguousarray(v)).to(dev) for v in asm.matrices())
    o1, o2 = out(), out()
    h1.setup_solve(Pxs, Axs, q, l, u, *o1)
    qb, lb, ub = (torch.from_numpy(np.ascontiguousarray(v)).to(dev) for v in (qh, lh, uh))
    Pb, Ab = (torch.from_numpy(np.ascontiguousarray(v)).to(dev) for v in (Px, Ax))
    h2.setup_solve(Pb, Ab, qb, lb, ub, *o2)
    torch.cuda.synchronize()
    for a, c in zip(o1, o2):
        assert torch.equal(a, c)
    assert (o1[2] == 1).all()
