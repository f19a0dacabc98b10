"""Host QP assembly (python-mpc_amd/osqp_amd/mpc.py) vs data captured from the
reference's own builders (tests/golden/make_golden.py).  CPU only."""
import json

import numpy as np
import pytest

from osqp_amd import mpc


def dense(M):
    return np.asarray(M.todense())


def test_slack_setup_matches_reference(golden):
    g = golden("slack_n20.npz")
    P, q, A, l, u = mpc.slack_qp(20, np.array([0., 0., 5 * np.pi / 180, 3., 0.]))
    assert np.array_equal(dense(P), dense(g["P"]))
    assert np.array_equal(dense(A), dense(g["A"]))
    assert np.array_equal(q, g["q"]) and np.array_equal(l, g["l"]) and np.array_equal(u, g["u"])
    assert json.loads(str(g["settings"])) == {"warm_start": True}


@pytest.mark.parametrize("k,regime", [(0, 0), (1, 1), (2, 0)])
def test_slack_update_regimes(golden, k, regime):
    """loop steps 0 / 401 / 901 (slack script :158-172); x0 is the (stub) open-loop state."""
    g = golden("slack_n20.npz")
    l_ref, u_ref = g["upd_l"][k], g["upd_u"][k]
    x0 = -l_ref[:5]
    _, q, _, l, u = mpc.slack_qp(20, x0, regime=regime)
    assert np.array_equal(q, g["upd_q"][k])
    assert np.array_equal(l, l_ref) and np.array_equal(u, u_ref)


def test_vanilla_matches_reference(golden):
    g = golden("vanilla_n20.npz")
    for t in range(g["q"].shape[0]):
        P, q, A, l, u = mpc.vanilla_qp(g["Ad"], g["Bd"], np.zeros(4), g["x0"][t], np.zeros((4, 21)), g["Q"], g["Q"],
                                       g["R"], 20, g["xmin"], g["xmax"], g["umin"], g["umax"])
        assert np.array_equal(dense(P), dense(g["P"]))
        assert np.array_equal(dense(A), dense(g["A"]))
        assert np.array_equal(q, g["q"][t]) and np.array_equal(l, g["l"][t]) and np.array_equal(u, g["u"][t])


def test_incremental_dynamic_matches_reference(golden):
    g = golden("dyn_incr_n50.npz")
    for t in range(g["q"].shape[0]):
        P, q, A, l, u = mpc.incremental_qp(list(g["Ad"][t]), list(g["Bd"][t]), list(g["gd"][t]), g["xt0"][t],
                                           g["Xr"][t], g["Q"], g["QN"], g["R"], 50, g["xmin_t"], g["xmax_t"],
                                           g["del_umin"], g["del_umax"])
        Pr = g["P"].copy(); Pr.data = g["Px"][t]
        Ar = g["A"].copy(); Ar.data = g["Ax"][t]
        assert np.allclose(dense(P), dense(Pr), rtol=0, atol=0)
        assert np.allclose(dense(A), dense(Ar), rtol=1e-15, atol=0)
        assert np.allclose(q, g["q"][t], rtol=1e-15, atol=0)
        assert np.array_equal(l, g["l"][t]) and np.array_equal(u, g["u"][t])


def test_kinematic_incremental_matches_reference(golden):
    g = golden("kin_incr_n40.npz")
    P, q, A, l, u = mpc.incremental_qp(list(g["Ad"]), list(g["Bd"]), list(g["gd"]), g["xt0"], g["Xr"],
                                       np.diag([50.0, 50.0, 10.0, 50.0]), np.diag([1000.0, 1000.0, 100.0, 1000.0]),
                                       np.diag([100., 100.]), 40,
                                       np.array([-np.inf, -np.inf, -100., -2 * np.pi, -np.deg2rad(15), -3.]),
                                       np.array([np.inf, np.inf, 100., 2 * np.pi, np.deg2rad(15), 1.]),
                                       np.array([-np.deg2rad(0.5), -0.5]), np.array([np.deg2rad(0.5), 0.5]))
    assert np.allclose(dense(P), dense(g["P"]), rtol=0, atol=0)
    assert np.allclose(dense(A), dense(g["A"]), rtol=1e-15, atol=0)
    assert np.allclose(q, g["q"], rtol=1e-15, atol=0)
    assert np.array_equal(l, g["l"]) and np.array_equal(u, g["u"])


def test_linearisation_matches_reference(golden):
    g = golden("linearise.npz")
    veh = mpc.VehicleParams(dt=float(g["dt"]))
    Ad, Bd, gd = mpc.linearise_dynamics(veh, g["x"], g["u"])
    assert np.allclose(Ad, g["Ad"], rtol=1e-13, atol=1e-15)
    assert np.allclose(Bd, g["Bd"], rtol=1e-13, atol=1e-15)
    assert np.allclose(gd, g["gd"], rtol=1e-12, atol=1e-13)


@pytest.mark.parametrize("cfg", [2, 3, 5])
def test_make_batch_instances_are_reference_layouts(cfg):
    """Each synthetic instance equals the single-instance builder at its own inputs."""
    b = mpc.make_batch(cfg, B=3)
    assert b["Px"].shape == (3, b["P"].nnz) and b["Ax"].shape == (3, b["A"].nnz)
    for t in range(3):
        A = b["A"].copy(); A.data = b["Ax"][t].copy()
        P = b["P"].copy(); P.data = b["Px"][t].copy()
        if cfg == 2:
            x0 = -b["l"][t][:4]
            P2, q2, A2, l2, u2 = mpc.vanilla_qp(mpc.LATERAL_AD, mpc.LATERAL_BD, np.zeros(4), x0, np.zeros((4, 21)),
                                                mpc.VANILLA_Q, mpc.VANILLA_Q, mpc.VANILLA_R, 20, mpc.VANILLA_XMIN,
                                                -mpc.VANILLA_XMIN, -mpc.VANILLA_UMAX, mpc.VANILLA_UMAX)
        elif cfg == 3:
            x0 = -b["l"][t][:5]
            regime = 1 if b["l"][t][5 * 21 + 3] == 2.0 else 0
            P2, q2, A2, l2, u2 = mpc.slack_qp(20, x0, regime=regime)
        else:
            continue
        assert np.array_equal(dense(P), dense(P2)) and np.array_equal(dense(A), dense(A2))
        assert np.array_equal(b["q"][t], q2) and np.array_equal(b["l"][t], l2) and np.array_equal(b["u"][t], u2)


def test_make_batch_dynamic_consistent():
    """cfg 5: instance values placed in the shared pattern equal the LTV builder's matrix."""
    b = mpc.make_batch(5, B=2, N=10)
    veh = mpc.VehicleParams(dt=0.05)
    # rebuild instance 0 from its own rollout
    rng = np.random.default_rng(5)
    xs = np.zeros((2, 6)); xs[:, 2] = rng.uniform(-np.pi / 8, np.pi / 8, 2); xs[:, 3] = rng.uniform(5, 25, 2)
    xs[:, 4] = rng.uniform(-.5, .5, 2); xs[:, 5] = rng.uniform(-.2, .2, 2)
    us = np.stack([np.deg2rad(rng.uniform(-5, 5, 2)), rng.uniform(-1, 1, 2)], axis=1)
    Ads, Bds, gds = [], [], []
    xk = xs.copy()
    for k in range(10):
        Ad, Bd, gd = mpc.linearise_dynamics(veh, xk, us)
        Ads.append(Ad[0]); Bds.append(Bd[0]); gds.append(gd[0])
        xk = np.einsum("bij,bj->bi", Ad, xk) + np.einsum("bij,bj->bi", Bd, us) + gd
    yoff = rng.uniform(-4, 4, 2)
    Xr = np.zeros((6, 11)); Xr[0] = np.arange(11) * 0.5; Xr[1] = yoff[0]; Xr[3] = 10.0
    P2, q2, A2, l2, u2 = mpc.incremental_qp(Ads, Bds, gds, np.concatenate([xs[0], us[0]]), Xr, mpc.DYN_Q, mpc.DYN_QN,
                                            mpc.DYN_R, 10, mpc.DYN_XMIN_T, mpc.DYN_XMAX_T, mpc.DYN_DUMIN,
                                            -mpc.DYN_DUMIN)
    A = b["A"].copy(); A.data = b["Ax"][0].copy()
    assert np.array_equal(dense(A), dense(A2))
    assert np.allclose(b["q"][0], q2, rtol=1e-15, atol=0)
    assert np.array_equal(b["l"][0], l2) and np.array_equal(b["u"][0], u2)


@pytest.mark.parametrize("layout,cfg", [("vanilla", 2), ("slack", 3)])
def test_lateral_affine_map_reproduces_the_builders(layout, cfg):
    """F1 for the lateral layouts (osqp_amd.mpc_device.AffineMap, evaluated here with the
    device kernel's arithmetic): q, l, u of seeded batches -- random x0, xr and bound
    regimes -- equal the host builders' (mpc.py, themselves equal to the reference's
    assembly: test_*_golden above) bit for bit, and make_batch's vectors from its theta."""
    from osqp_amd.mpc_device import AffineMap, lateral_builder
    N = 20
    build, nparam, nreg, (P, A) = lateral_builder(layout, N)
    amap = AffineMap(build, nparam, nreg)
    assert amap.T <= 1  # diagonal weights: every entry one product (q = -Q xr, l = u = -x0) or a constant
    rng = np.random.default_rng(9)
    theta = rng.normal(size=(6, nparam)) * 3
    reg = rng.integers(0, nreg, 6)
    q, l, u = amap.evaluate(theta, reg)
    for b in range(6):
        qr, lr, ur = build(theta[b], int(reg[b]))
        assert np.array_equal(q[b], qr) and np.array_equal(l[b], lr) and np.array_equal(u[b], ur)
    bt = mpc.make_batch(cfg, B=16, seed=4)
    q, l, u = amap.evaluate(bt["theta"], bt["regime"])
    assert np.array_equal(q, bt["q"]) and np.array_equal(l, bt["l"]) and np.array_equal(u, bt["u"])


def test_lateral_affine_map_on_reference_fixtures(golden):
    """The same map against the vectors the reference's own code built: the slack script's
    update(q, l, u) of loop steps 0, 401 and 901 (x~0 from their l = u rows, regime by the
    script's schedule :158-172) and mpc_kinematics.mpc's four captured QPs."""
    from osqp_amd.mpc_device import AffineMap, lateral_builder
    g = golden("slack_n20.npz")
    amap = AffineMap(*lateral_builder("slack", 20)[:3])
    for k, step in enumerate(g["steps"]):
        theta = np.concatenate([-g["upd_l"][k][:5], np.zeros(4)])
        reg = 0 if step <= 400 or step > 900 else 1
        q, l, u = amap.evaluate(theta[None], [reg])
        assert np.array_equal(q[0], g["upd_q"][k]) and np.array_equal(l[0], g["upd_l"][k])
        assert np.array_equal(u[0], g["upd_u"][k])
    g = golden("vanilla_n20.npz")
    amap = AffineMap(*lateral_builder("vanilla", 20)[:3])
    for t in range(g["x0"].shape[0]):
        theta = np.concatenate([g["x0"][t], np.zeros(4 * 21)])
        q, l, u = amap.evaluate(theta[None])
        assert np.array_equal(q[0], g["q"][t]) and np.array_equal(l[0], g["l"][t]) and np.array_equal(u[0], g["u"][t])
