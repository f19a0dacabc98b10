"""Parity of the MI355X solver (libmpcqp.so, through the osqp.OSQP-shaped host
API) with the CPU oracle (OSQP 0.6 restatement) on the same inputs.

Tolerance (BASELINE.json north_star): per instance ||u* - u*_ref||_inf < 1e-4 at
the same ADMM eps; in practice the iterates agree to ~1e-9 because only the
linear-system method differs (block-tridiagonal reduced KKT vs quasi-definite
LDL'), so we also require equal status and iteration counts for >= 99% of
instances and a 1e-6 bound on the whole primal vector (relative to its scale).
"""
import json

from types import SimpleNamespace

import numpy as np
import pytest

import pyoracle
from osqp_amd import OSQP, OSQPBatch, mpc
from parity import check_agreement

pytestmark = pytest.mark.gpu

U_TOL = 1e-4


def _settings(g):
    s = json.loads(str(g["settings"]))
    s.pop("verbose", None)
    return s


def _cmp_single(P, q, A, l, u, settings, u_slice):
    o = pyoracle.OSQP()
    o.setup(P, q, A, l, u, **settings)
    ro = o.solve()
    g = OSQP()
    g.setup(P, q, A, l, u, **settings)
    rg = g.solve()
    assert rg.info.status == ro.info.status
    assert rg.info.iter == ro.info.iter
    scale = max(1.0, np.abs(ro.x).max())
    assert np.abs(rg.x - ro.x).max() < 1e-6 * scale
    assert np.abs(rg.x[u_slice] - ro.x[u_slice]).max() < U_TOL
    assert np.abs(rg.y - ro.y).max() < 1e-5 * max(1.0, np.abs(ro.y).max())
    return ro, rg


def test_vanilla_golden(golden):
    g = golden("vanilla_n20.npz")
    for t in range(g["q"].shape[0]):
        _cmp_single(g["P"], g["q"][t], g["A"], g["l"][t], g["u"][t], _settings(g), slice(84, 104))


def test_slack_golden_and_updates(golden):
    """setup + update(q,l,u) + solve with warm start (slack script :121,237,248)."""
    g = golden("slack_n20.npz")
    s = _settings(g)
    o = pyoracle.OSQP(); o.setup(g["P"], g["q"], g["A"], g["l"], g["u"], **s)
    d = OSQP(); d.setup(g["P"], g["q"], g["A"], g["l"], g["u"], **s)
    for k in range(-1, 3):
        if k >= 0:
            o.update(q=g["upd_q"][k], l=g["upd_l"][k], u=g["upd_u"][k])
            d.update(q=g["upd_q"][k], l=g["upd_l"][k], u=g["upd_u"][k])
        ro, rd = o.solve(), d.solve()
        assert rd.info.status == ro.info.status == "solved"
        assert rd.info.iter == ro.info.iter
        assert np.abs(rd.x - ro.x).max() < 1e-6 * max(1, np.abs(ro.x).max())
        assert np.abs(rd.x[105:125] - ro.x[105:125]).max() < U_TOL


def test_dynamic_incremental_golden(golden):
    g = golden("dyn_incr_n50.npz")
    for t in range(g["q"].shape[0]):
        P = g["P"].copy(); P.data = g["Px"][t].copy()
        A = g["A"].copy(); A.data = g["Ax"][t].copy()
        _cmp_single(P, g["q"][t], A, g["l"][t], g["u"][t], _settings(g), slice(408, 508))


def test_kinematic_incremental_golden(golden):
    g = golden("kin_incr_n40.npz")
    _cmp_single(g["P"], g["q"], g["A"], g["l"], g["u"], _settings(g), slice(246, 326))


@pytest.mark.parametrize("name,nu", [("kin_ltv_n40.npz", 2), ("kin_corridor_n30.npz", 2), ("dyn_ltv_n30.npz", 2),
                                     ("incr_func_n40.npz", 2)])
def test_reference_builder_qps(golden, name, nu):
    """QPs of the reference's other builders, captured from its own code (make_golden.py):
    mpc_kinematics_pred_matrix.mpc__ (LTV), mpc_kinematics.mpc_ (per-stage corridor bounds),
    mpc_dynamics.mpc (LTV dynamic model), mpc_incre_kine_func.mpc_increment -- each with the
    settings its call site passes.  The controls are the last N nu variables."""
    g = golden(name)
    n = g["P"].shape[0]
    N = int(name.split("_n")[1].split(".")[0])
    _cmp_single(g["P"], g["q"], g["A"], g["l"], g["u"], _settings(g), slice(n - N * nu, n))


def _batch_parity(b, settings, nthreads=16, min_match=1.0, rg=None, label=None, x0=None, y0=None):
    """Device vs oracle over batch b: tests/parity.py::check_agreement (agreement fractions
    recorded; every disagreeing instance held to OSQP's termination test and compared with
    the optimum, the oracle at eps 1e-9)."""
    ws = {} if x0 is None else dict(x0=x0, y0=y0)
    bo = pyoracle.solve_batch(b["P"], b["A"], b["Px"], b["q"], b["Ax"], b["l"], b["u"], nthreads=nthreads,
                              **ws, **settings)

    def tight(d):
        w = {} if x0 is None else dict(x0=x0[d], y0=y0[d])
        return pyoracle.solve_batch(b["P"], b["A"], b["Px"][d], b["q"][d], b["Ax"][d], b["l"][d], b["u"][d],
                                    nthreads=nthreads, **w,
                                    **dict(settings, eps_abs=1e-9, eps_rel=1e-9, max_iter=200000)).x
    if rg is None:
        bg = OSQPBatch()
        bg.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **settings)
        rg = bg.solve()
    label = label or f"cfg{b.get('cfg', '?')} B={b['Px'].shape[0]}"
    y = getattr(rg, "y", None)
    du = check_agreement(label, b, rg.x, y, rg.status_val, rg.iter, bo, min_match=min_match,
                         tight=tight if settings.get("eps_abs", 1e-3) > 1e-8 else None)
    return du, rg, bo


def test_cfg2_batch_1024():
    b = mpc.make_batch(2, B=1024)
    du, rg, bo = _batch_parity(b, dict(warm_start=True))
    assert (rg.status_val == 1).all()


def test_cfg3_batch_sample():
    b = mpc.make_batch(3, B=512)
    du, rg, bo = _batch_parity(b, dict(warm_start=True))


def test_cfg5_batch_sample():
    # (cold long-horizon solves of ~400 iterations: a count may part by one check interval --
    # the reduced KKT's rounding, DESIGN.md §3 -- on an instance; it is held to the termination
    # test and the eps bound instead)
    b = mpc.make_batch(5, B=64)
    du, rg, bo = _batch_parity(b, dict(polish=False, warm_start=False), min_match=0.98)


def test_invalid_bounds_raise():
    b = mpc.make_batch(2, B=2)
    l = b["l"].copy(); l[1, 10] = b["u"][1, 10] + 1.0
    with pytest.raises(ValueError):
        OSQPBatch().setup(b["P"], b["q"], b["A"], l, b["u"])


def test_primal_infeasible_status():
    """x <= -1 and x >= 1 on one variable: OSQP reports 'primal infeasible'."""
    import scipy.sparse as sp
    P = sp.csc_matrix(np.eye(2)); q = np.zeros(2)
    A = sp.csc_matrix(np.array([[1.0, 0.0], [1.0, 0.0], [0.0, 1.0]]))
    l = np.array([-np.inf, 1.0, -1.0]); u = np.array([-1.0, np.inf, 1.0])
    o = pyoracle.OSQP(); o.setup(P, q, A, l, u); ro = o.solve()
    g = OSQP(); g.setup(P, q, A, l, u); rg = g.solve()
    assert ro.info.status == "primal infeasible"
    assert rg.info.status == ro.info.status and rg.info.iter == ro.info.iter
    assert np.allclose(rg.prim_inf_cert, ro.prim_inf_cert, atol=1e-8)


def test_dual_infeasible_status():
    """min -x s.t. x >= 0 (unbounded): 'dual infeasible'."""
    import scipy.sparse as sp
    P = sp.csc_matrix((2, 2)); q = np.array([-1.0, 0.0])
    A = sp.csc_matrix(np.eye(2)); l = np.array([0.0, -1.0]); u = np.array([np.inf, 1.0])
    o = pyoracle.OSQP(); o.setup(P, q, A, l, u); ro = o.solve()
    g = OSQP(); g.setup(P, q, A, l, u); rg = g.solve()
    assert ro.info.status == "dual infeasible"
    assert rg.info.status == ro.info.status and rg.info.iter == ro.info.iter


def _slack_script_loop(osqp_mod, nsim=1500, N=20, states=None, **settings):
    """BASELINE.json configs[0]: vehicle_lateral_mpc_slack_increment.py as written, at N = 20
    (the script ships N = 100, :14; test_slack_script_default_horizon covers that size).
    setup once with warm_start (:118-121), then every step exactly the script's calls:
    update(q=, l=, u=) with the rebuilt vectors (:201-229, :237) under the bound schedule
    i <= 400 / <= 900 / else (:158-172), solve (:248), raise unless 'solved' (:252-253),
    du_0 = x[(N+1) nx] (:256), the plant x0 = A~ x0 + B~ du_0 (:257), the slack of e_y
    (:259), then update(l=, u=) with the new initial state (:267-269).  Returns per step
    (du_0, iterations, slack) and the plant states.  `states`: drive the loop along these
    plant states instead of its own (the solver still warm-starts from its own solutions).
    `settings`: passed to setup() besides the script's warm_start=True (diagnostics only)."""
    x0 = np.array([0.0, 0.0, 5 * mpc.DEG, 3.0, 0.0])                         # :27
    P, q, A, l, u = mpc.slack_qp(N, x0)
    prob = osqp_mod.OSQP()
    prob.setup(P, q, A, l, u, warm_start=True, **settings)                   # :121
    At, Bt = mpc.augment(mpc.LATERAL_AD, mpc.LATERAL_BD)
    nx = At.shape[0]
    out, xs = [], [x0]
    for i in range(nsim):
        regime = 0 if i <= 400 else (1 if i <= 900 else 0)                   # :158-172
        _, q_new, _, l_new, u_new = mpc.slack_qp(N, x0, regime=regime)       # :201-229 (xr = 0, :126-129)
        prob.update(q=q_new, l=l_new, u=u_new)                               # :237
        res = prob.solve()                                                   # :248
        if res.info.status != "solved":                                      # :252-253
            raise ValueError("OSQP did not solve the problem!")
        del_ctrl = res.x[(N + 1) * nx:(N + 1) * nx + 1]                      # :256
        x0 = At @ x0 + Bt @ del_ctrl                                         # :257
        if states is not None:
            x0 = states[i + 1]
        xs.append(x0)
        slack = res.x[-(N + 1) * nx:][3]                                     # :259
        out.append((del_ctrl[0], res.info.iter, slack))
        l_new[:nx] = -x0                                                     # :267-269
        u_new[:nx] = -x0
        prob.update(l=l_new, u=u_new)
    return np.array(out), np.array(xs)


def test_slack_script_configs0_1500_steps():
    """configs[0] through the `import osqp` drop-in (python-mpc_amd/shim/osqp.py): the
    script's 1500-step closed loop, every call as the script makes it, against the oracle.
    At N = 20 the loop is poorly damped (e_y swings to +-200 m and the slack carries it),
    so rounding-level differences in du_0 grow through the plant: run free, the device's
    and the oracle's trajectories part after ~1000 steps.  The device loop is therefore
    driven along the oracle's plant states (warm-starting from its own solutions).  Bar:
    iteration counts as below; du_0 within the north-star 1e-4 while the state
    stays moderate (the first 800 steps, |x0| < 135); for the first 1000 steps within a tenth
    of OSQP's own termination tolerance eps_abs + eps_rel |x0| at that step's scale, and at
    every step within that tolerance itself (both CPU and device results are OSQP solutions
    only to that tolerance; the full-plan device solve, MPCQP_ELIM=0, reaches 0.75 of it in
    the late steps, profiles/r3_diag_configs0.txt, as the eliminated-slack one does since
    the round-3 phase-A accumulation order).  Past
    |x0| ~ 100 the warm-started solve chain itself amplifies rounding: the oracle against
    itself with the states perturbed by 1e-14 (relative) moves du_0 by 3e-4
    (tools/diag_configs0.py; profiles/r3_diag_configs0.txt).

    Iteration counts: equal at every step of the first 1000; past that, different at no
    more than 1 % of the loop's steps (15), each by one termination-check interval (25).  The
    three-solver record (tools/diag_configs0_three.py, profiles/r4s2_configs0/): from identical
    starts -- each step's QP warm-started from the oracle's previous solution -- the oracle,
    the dense numpy restatement and the device take the same count at 1496 of 1499 steps, and
    the device's x is as close to the oracle's as the restatement's (median 1.1e-13, p90 6e-12
    relative, against 1.1e-13 / 9e-12).  In this driven loop each solver warm-starts from its own
    previous solutions, and the chains drift apart at rounding level: the restatement's happens
    to keep every count; the device's parts at steps 1051 and 1073 (100 -> 125, 50 -> 25; at
    1073 the restatement's own decision was 0.9 % from the threshold), and with round 3's phase-A
    summation on the slack instantiation at 1039-1041 and 1074 instead (margins 0.09 %, 3.9 %,
    9.6 %, 0.8 %) -- so which late steps flip follows the rounding order, not a wrong decision.
    That summation order was not restored: it cost 1.6 % on cfg 3 (same-box A/B,
    profiles/r4s2_configs0/el_single_chain/).  du_0 stays within a tenth of OSQP's tolerance at all of them."""
    import importlib.util
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("osqp", os.path.join(root, "python-mpc_amd", "shim", "osqp.py"))
    shim = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(shim)
    o, xo = _slack_script_loop(pyoracle)
    g, _ = _slack_script_loop(shim, states=xo)
    assert g.shape == (1500, 3)
    mism = np.flatnonzero(g[:, 1] != o[:, 1])
    assert mism.size == 0 or mism.min() >= 1000, mism[:10]
    assert mism.size <= 15, mism  # <= 1 % of the 1500 steps
    assert np.all(np.abs(g[mism, 1] - o[mism, 1]) == 25), (mism, g[mism, 1], o[mism, 1])
    d = np.abs(g[:, 0] - o[:, 0])
    tol = 1e-3 + 1e-3 * np.abs(xo[:-1]).max(axis=1)  # eps_abs + eps_rel |x0|_inf per step
    assert d[:800].max() < U_TOL, d[:800].max()
    assert np.all(d[:1000] <= 0.1 * tol[:1000]), np.max(d[:1000] / tol[:1000])
    assert np.all(d <= tol), np.max(d / tol)
    ds = np.abs(g[:, 2] - o[:, 2])
    assert np.all(ds[:1000] <= 0.1 * tol[:1000]) and np.all(ds <= tol), np.max(ds / tol)


def test_slack_script_configs0_free_running():
    """configs[0] free-running: the device's closed loop on its own plant trajectory (not driven
    along the oracle's states), every call as the script makes it, against the oracle's own
    free-running loop.  Two correct implementations of OSQP 0.6 part in this poorly damped loop:
    the dense numpy restatement against the oracle (tools/diag_configs0_three.py --loops,
    profiles/r4s2_configs0/three_loops.txt) keeps du_0 within 1e-4 up to step 801 and its
    iteration counts equal up to step 1050, then its trajectory and the oracle's separate (11
    steps one check interval apart, du_0 up to 1.8e-2, the e_y envelope 1.6 % wider).  The
    device's bar is the one that restatement meets: all 1500 steps solved (the script raises
    otherwise, :252-253); du_0 within the north star's 1e-4 for the first 800 steps; equal
    iteration counts for the first 1000; past that -- two different trajectories -- at most
    2 % of the steps with a different count; and the plant's per-state envelope max_k |x_k|
    within 3 % of the oracle's
    (measured: du_0 within 1e-4 up to step 1036, first count mismatch at 1039, envelope 1.4 %)."""
    import importlib.util
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("osqp", os.path.join(root, "python-mpc_amd", "shim", "osqp.py"))
    shim = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(shim)
    o, xo = _slack_script_loop(pyoracle)
    g, xg = _slack_script_loop(shim)
    assert g.shape == (1500, 3)
    d = np.abs(g[:, 0] - o[:, 0])
    assert d[:800].max() < U_TOL, d[:800].max()
    mism = np.flatnonzero(g[:, 1] != o[:, 1])
    assert mism.size == 0 or mism.min() >= 1000, mism[:10]
    assert mism.size <= 30, mism
    env_o, env_g = np.abs(xo).max(axis=0), np.abs(xg).max(axis=0)
    assert np.all(np.abs(env_g - env_o) <= 0.03 * env_o + 1e-9), (env_g, env_o)


def _stage_shift(v, N, nxa, nu, groups):
    """One-stage shift of incremental-layout iterates (mpcqp_incr_warm_shift_device)."""
    B = v.shape[0]
    out = []
    for g in range(groups):
        blk = v[:, g * (N + 1) * nxa:(g + 1) * (N + 1) * nxa].reshape(B, N + 1, nxa)
        out.append(np.concatenate([blk[:, 1:], blk[:, -1:]], 1).reshape(B, -1))
    du = v[:, groups * (N + 1) * nxa:].reshape(B, N, nu)
    out.append(np.concatenate([du[:, 1:], du[:, -1:]], 1).reshape(B, -1))
    return np.concatenate(out, 1)


def test_cfg5_warm_started_batch():
    """cfg 5 as bench.py times it: warm start from the cold solution
    shifted one stage; device and oracle start from the same (x, y)."""
    b = mpc.make_batch(5, B=64)
    s = {k: v for k, v in b["settings"].items() if k != "verbose"}
    r0 = pyoracle.solve_batch(b["P"], b["A"], b["Px"], b["q"], b["Ax"], b["l"], b["u"], nthreads=16, **s)
    xs, ys = _stage_shift(r0.x, b["N"], 8, 2, 1), _stage_shift(r0.y, b["N"], 8, 2, 2)
    bo = pyoracle.solve_batch(b["P"], b["A"], b["Px"], b["q"], b["Ax"], b["l"], b["u"], nthreads=16, x0=xs, y0=ys,
                              **s)
    bg = OSQPBatch()
    bg.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
    bg.warm_start(x=xs, y=ys)
    rg = bg.solve()
    # (warm-started long-horizon solves: see test_cfg5_batch_sample on the 0.95 bar)
    _batch_parity(b, s, min_match=0.95, rg=rg, label="cfg5 B=64 warm", x0=xs, y0=ys)
    assert bo.iter.mean() < r0.iter.mean()


@pytest.mark.parametrize("name", ["vanilla_n20.npz", "slack_n20.npz", "dyn_incr_n50.npz", "kin_incr_n40.npz"])
def test_polish_matches_oracle(golden, name):
    """polish=True (OSQP 0.6 polish.c): same accept / reject decision
    as the oracle; an accepted polished point is the reduced KKT solution, so x and y
    agree to far below the ADMM tolerance."""
    g = golden(name)
    if g["q"].ndim == 2:
        P = g["P"].copy(); A = g["A"].copy()
        if "Px" in g:
            P.data = g["Px"][0].copy(); A.data = g["Ax"][0].copy()
        q, l, u = g["q"][0], g["l"][0], g["u"][0]
    else:
        P, A, q, l, u = g["P"], g["A"], g["q"], g["l"], g["u"]
    s = dict(_settings(g), polish=True)
    o = pyoracle.OSQP(); o.setup(P, q, A, l, u, **s); ro = o.solve()
    d = OSQP(); d.setup(P, q, A, l, u, **s); rd = d.solve()
    assert rd.info.status == ro.info.status and rd.info.iter == ro.info.iter
    assert rd.info.status_polish == ro.info.status_polish
    scale = max(1.0, np.abs(ro.x).max())
    tol = 1e-8 if ro.info.status_polish == 1 else 1e-6
    assert np.abs(rd.x - ro.x).max() < tol * scale
    assert np.abs(rd.y - ro.y).max() < 100 * tol * max(1.0, np.abs(ro.y).max())
    if ro.info.status_polish == 1:
        assert rd.info.pri_res < 1e-9 and rd.info.dua_res < 1e-9


def test_polish_batch_cfg2():
    b = mpc.make_batch(2, B=256)
    bo = pyoracle.solve_batch(b["P"], b["A"], b["Px"], b["q"], b["Ax"], b["l"], b["u"], nthreads=16,
                              warm_start=True, polish=True)
    bg = OSQPBatch()
    bg.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], warm_start=True, polish=True)
    rg = bg.solve()
    assert (rg.status_polish == 1).mean() > 0.9
    same = rg.iter == bo.iter
    assert same.mean() >= 0.99
    du = np.abs(rg.x[:, b["u_block"]] - bo.x[:, b["u_block"]]).max(axis=1)
    assert np.all(du[same] < 1e-6), du.max()


@pytest.mark.parametrize("variant,cfg,B", [(11, 3, 256), (12, 5, 64), (10, 2, 1024), (17, 2, 1024), (0, 2, 512),
                                             (7, 2, 512)])
def test_alternative_kernel_variants(monkeypatch, variant, cfg, B):
    """Kernel instantiations that are not the default choice for a plan stay exact:
    the 512-thread two-sided kernel on the slack layout (variant 11), the long-horizon
    kernel on cfg 5 (12), the two-wave kernel (10, the default before the four-wave one)
    and the four-wave kernel (17) on cfg 2, the 256-thread register-factor kernels with the
    three-phase (0) and the sweep (7) solve on cfg 2, selected with the MPCQP_VARIANT override."""
    monkeypatch.setenv("MPCQP_VARIANT", str(variant))
    b = mpc.make_batch(cfg, B=B)
    settings = dict(warm_start=True) if cfg == 3 else dict(polish=False, warm_start=False)
    _batch_parity(b, settings, min_match=0.98 if cfg == 5 else 1.0)  # (cfg 5: test_cfg5_batch_sample)


EXPERIMENTAL = [(14, 3, 256), (8, 2, 256), (16, 2, 256), (18, 3, 256), (15, 5, 64), (19, 2, 1024)]


def test_experimental_kernel_variants(tmp_path):
    """The variants measured and not taken are built only into the exp
    library (python-mpc_amd/csrc/Makefile, MPCQP_EXPERIMENTAL): the two-wave two-sided
    kernel on the slack layout (14), the one-wave kernel (8) and the dense-inverse kernel
    (16) on cfg 2, the eight-wave kernel (18) on the slack layout, the 256-thread twisted
    long-horizon kernel (15) on cfg 5, the one-instance-per-CU latency kernel (19,
    solve_heavy.hip: 512 threads, M = K^-1 in registers) on the whole cfg-2 batch.  They stay exact against
    the oracle, solved in a child process under MPCQP_BUILD=exp; and the production
    library refuses them (MPCQP_VARIANT=v does not fit)."""
    import build_cases
    sets = {2: dict(polish=False, warm_start=False), 3: dict(warm_start=True), 5: dict(polish=False, warm_start=False)}
    specs = [("batch", f"v{v}", cfg, B, str(v), sets[cfg]) for v, cfg, B in EXPERIMENTAL]
    got = build_cases.in_build("exp", specs, tmp_path / "exp.npz")
    for v, cfg, B in EXPERIMENTAL:
        assert int(got[f"v{v}_variant"]) == v
        rg = SimpleNamespace(x=got[f"v{v}_x"], y=got[f"v{v}_y"], iter=got[f"v{v}_iter"],
                             status_val=got[f"v{v}_status_val"])
        _batch_parity(mpc.make_batch(cfg, B=B), sets[cfg], rg=rg, min_match=0.98 if cfg == 5 else 1.0,
                      label=f"exp variant {v}, cfg{cfg} B={B}")


def test_dense_inverse_form(tmp_path):
    """The four-wave kernel's dense-inverse form (MPCQP_DENSE_W4=1 in the experimental build:
    M^-1 = L' D L formed after each factorisation, solve_wave.hip DK, on the planner's balanced
    blocks) against the oracle, in a child process (the switch is read once per process): cfg 2 with the
    workload's settings, and with a termination check after every iteration -- the rows of
    M^-1 must survive every run boundary (a form that kept them in registers across the
    check went wrong from the fifth check on)."""
    import build_cases
    sets = {"dflt": dict(polish=False, warm_start=False),
            "ck1": dict(polish=False, warm_start=False, check_termination=1, max_iter=60)}
    specs = [("batch", k, 2, 1024, None, s) for k, s in sets.items()]
    got = build_cases.in_build("exp", specs, tmp_path / "dk.npz", extra_env={"MPCQP_DENSE_W4": "1"})
    for k, s in sets.items():
        rg = SimpleNamespace(x=got[f"{k}_x"], y=got[f"{k}_y"], iter=got[f"{k}_iter"], status_val=got[f"{k}_status_val"])
        _batch_parity(mpc.make_batch(2, B=1024), s, rg=rg, label=f"cfg2 B=1024 dense-inverse form ({k})")


def test_long_horizon_interface_form(tmp_path):
    """The long-horizon kernel's interface form of the two-sided solve (solve_big.hip::iface_solve,
    experimental build, MPCQP_BIG_FORM=iface, read once per process: the amax / bmax-row recurrences run by one
    wave per chain, everything else between four barriers) against the oracle on cfg 5, in a
    child process; and the same batch through the default twisted sweep agrees with it."""
    import build_cases
    s = dict(polish=False, warm_start=False)
    got = build_cases.in_build("exp", [("batch", "if", 5, 64, None, s)], tmp_path / "if.npz",
                               extra_env={"MPCQP_BIG_FORM": "iface"})
    assert int(got["if_variant"]) == 12
    b = mpc.make_batch(5, B=64)
    rg = SimpleNamespace(x=got["if_x"], y=got["if_y"], iter=got["if_iter"], status_val=got["if_status_val"])
    _batch_parity(b, s, rg=rg, min_match=0.98, label="cfg5 B=64 interface form")
    h = OSQPBatch()
    h.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
    r = h.solve()
    same = r.iter == rg.iter
    assert same.mean() >= 0.9 and np.array_equal(r.status_val, rg.status_val)
    assert np.abs(r.x[same] - rg.x[same]).max() < 1e-6 * max(1.0, np.abs(r.x).max())


@pytest.mark.parametrize("variant", [v for v, _, _ in EXPERIMENTAL])
def test_production_library_refuses_experimental_variants(monkeypatch, variant):
    cfg = next(c for v, c, _ in EXPERIMENTAL if v == variant)
    monkeypatch.setenv("MPCQP_VARIANT", str(variant))
    b = mpc.make_batch(cfg, B=4)
    with pytest.raises(Exception, match="does not fit"):
        OSQPBatch().setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"])


@pytest.mark.parametrize("settings", [
    dict(max_iter=30),                                   # stops between checks: approximate final check
    dict(max_iter=60, check_termination=0),              # no termination checks at all
    dict(adaptive_rho=False),                            # fixed rho: one factorisation
    dict(adaptive_rho_interval=50),                      # rho updates between the default ones
    dict(alpha=1.0, rho=0.5, sigma=1e-4),                # non-default ADMM parameters
    dict(eps_abs=1e-5, eps_rel=1e-5),                    # tight tolerances: more iterations
    dict(scaling=0),                                     # no Ruiz equilibration
    dict(scaled_termination=True),                       # residuals in the scaled space
])
def test_settings_paths_match_oracle(settings):
    """Settings the reference never changes but osqp.OSQP accepts, each steering a
    different path of the two-wave kernel (check cadence, final approximate check,
    rho adaptation, unscaled / scaled residuals), against the oracle on a cfg-2
    batch; B = 96 is not a multiple of the residency round."""
    b = mpc.make_batch(2, B=96, seed=7)
    s = dict(warm_start=False, polish=False)
    s.update(settings)
    _batch_parity(b, s)


@pytest.mark.parametrize("cfg,B", [(3, 1), (3, 3), (2, 1), (2, 3)])
def test_tiny_batches(cfg, B):
    """Batches smaller than a wave of instances (one and three QPs), for the slack
    layout's register-sweep kernel and the vanilla layout's four-wave kernel."""
    b = mpc.make_batch(cfg, B=B, seed=11)
    _batch_parity(b, dict(warm_start=True), min_match=1.0)


def test_cfg2_warm_resolves_after_updates():
    """The four-wave kernel's warm path: the batch solved, then update(l, u) with the
    initial states moved (a receding-horizon step) and solved again from the previous
    x, z, y -- three times, each against the oracle doing the same."""
    b = mpc.make_batch(2, B=64, seed=5)
    s = dict(warm_start=True)
    P, A = b["P"], b["A"]
    dev = OSQPBatch()
    dev.setup(P, b["q"], A, b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
    orc = []
    for k in range(b["Px"].shape[0]):
        o = pyoracle.OSQP()
        Pk, Ak = P.copy(), A.copy()
        Pk.data, Ak.data = b["Px"][k].copy(), b["Ax"][k].copy()
        o.setup(Pk, b["q"][k], Ak, b["l"][k], b["u"][k], **s)
        orc.append(o)
    rng = np.random.default_rng(7)
    l, u = b["l"].copy(), b["u"].copy()
    for step in range(3):
        if step:
            x0 = -l[:, :4] + rng.uniform(-0.02, 0.02, (l.shape[0], 4))
            l[:, :4] = -x0
            u[:, :4] = -x0
            dev.update(l=l, u=u)
            for k, o in enumerate(orc):
                o.update(l=l[k], u=u[k])
        rd = dev.solve()
        ro = [o.solve() for o in orc]
        it = np.array([r.info.iter for r in ro])
        assert np.mean(rd.iter == it) >= 0.99
        same = rd.iter == it
        du = np.array([np.abs(rd.x[k, b["u_block"]] - ro[k].x[b["u_block"]]).max() for k in range(len(ro))])
        assert np.all(du[same] < U_TOL), du.max()


@pytest.mark.parametrize("cfg,B", [(2, 1024), (3, 1024), (5, 320)])
def test_longest_first_dispatch_is_result_neutral(monkeypatch, cfg, B):
    """kernels.hip::k_order reorders the solve kernel's workgroups by the previous
    solve's iteration counts.  One handle solves batch X (identity order; the order
    is then set from X's counts), then setup()+solve() batch Y in the reordered
    dispatch; that must be bit-identical to a handle that dispatches Y in identity
    order (MPCQP_DISPATCH=identity).  An instance the reordered launch skipped would
    still hold X's solution."""
    import torch
    from osqp_amd import DeviceBatch
    bx, by = mpc.make_batch(cfg, B=B, seed=101), mpc.make_batch(cfg, B=B, seed=202)
    s = {k: v for k, v in bx["settings"].items() if k != "verbose"}
    s.update(warm_start=False, polish=False)
    dev = torch.device("cuda", 0)
    n, m = bx["n"], bx["m"]

    def put(b):
        return [torch.from_numpy(np.ascontiguousarray(b[k])).to(dev) for k in ("Px", "Ax", "q", "l", "u")]

    def out():
        return (torch.empty((B, n), dtype=torch.float64, device=dev), torch.empty((B, m), dtype=torch.float64, device=dev),
                torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.int32, device=dev))

    X, Y = put(bx), put(by)
    lpt = DeviceBatch(bx["P"], bx["A"], B, device=0, **s)
    o1 = out()
    lpt.setup(*X); lpt.solve(*o1)
    lpt.setup(*Y); lpt.solve(*o1)
    lpt.synchronize()
    monkeypatch.setenv("MPCQP_DISPATCH", "identity")
    ref = DeviceBatch(bx["P"], bx["A"], B, device=0, **s)
    o0 = out()
    ref.setup(*Y); ref.solve(*o0)
    ref.synchronize()
    for a, b in zip(o1, o0):
        assert torch.equal(a, b)
    assert o1[3].max().item() > o1[3].min().item()  # the counts vary, so the order is not the identity


@pytest.mark.parametrize("cfg", [2, 3])
def test_fused_dispatch_order_matches_order_kernel(monkeypatch, cfg):
    """The order the solve kernel's last workgroup sorts (device_common.h::order_epilogue)
    against the separate sort kernel (kernels.hip::k_order, MPCQP_ORDER_KERNEL=1), read back
    through mpcqp_debug_dispatch_order after one solve of B = 1024 > resident slots: both
    are permutations that visit the instances by non-increasing iteration bucket
    (iter >> shift, 256 buckets) -- which fixes each bucket's set of instances, the order
    inside a bucket being the atomics' -- and neither is the identity it starts from.  A
    silent no-op or a differently keyed sort fails here, not only in timing."""
    import torch
    from osqp_amd import DeviceBatch
    B = 1024
    b = mpc.make_batch(cfg, B=B, seed=31)
    s = {k: v for k, v in b["settings"].items() if k != "verbose"}
    s.update(warm_start=False, polish=False)
    dev = torch.device("cuda", 0)
    X = [torch.from_numpy(np.ascontiguousarray(b[k])).to(dev) for k in ("Px", "Ax", "q", "l", "u")]
    max_iter = s.get("max_iter", 4000)
    shift = 0
    while (max_iter >> shift) >= 256:
        shift += 1
    keys = {}
    for mode in ("fused", "kernel"):
        if mode == "kernel":
            monkeypatch.setenv("MPCQP_ORDER_KERNEL", "1")
        d = DeviceBatch(b["P"], b["A"], B, device=0, **s)
        assert np.array_equal(d.dispatch_order(), np.arange(B))
        o = (torch.empty((B, b["n"]), dtype=torch.float64, device=dev),
             torch.empty((B, b["m"]), dtype=torch.float64, device=dev),
             torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.int32, device=dev))
        d.setup(*X)
        d.solve(*o)
        d.synchronize()
        it = o[3].cpu().numpy()
        order = d.dispatch_order()
        assert np.array_equal(np.sort(order), np.arange(B)), mode
        k = it[order] >> shift
        assert np.all(np.diff(k) <= 0), mode
        assert not np.array_equal(order, np.arange(B)), mode
        keys[mode] = (it, k)
    assert np.array_equal(keys["fused"][0], keys["kernel"][0])
    assert np.array_equal(keys["fused"][1], keys["kernel"][1])


@pytest.mark.parametrize("cfg,B", [(2, 200), (5, 24)])
def test_host_results_gather_matches_device_outputs(cfg, B):
    """A host-API solve of a small batch brings everything it returns back through one gather
    kernel into a device twin of the pinned staging layout and one copy (api.hip::
    mpcqp_solve_batch, kernels.hip::k_gather: x, y, the info, the certificates, the statuses,
    the polish flags as zeros).  The same batch through the device API (outputs written by the
    solve kernel into torch tensors, no gather) agrees bit for bit on x, y, status and
    iterations, and the info getters report the statuses and counts the kernel wrote."""
    import torch
    from osqp_amd import DeviceBatch
    b = mpc.make_batch(cfg, B=B, seed=23)
    s = {k: v for k, v in b["settings"].items() if k != "verbose"}
    s.update(warm_start=False, polish=False)
    h = OSQPBatch()
    h.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
    rh = h.solve()
    dev = torch.device("cuda", 0)
    X = [torch.from_numpy(np.ascontiguousarray(b[k])).to(dev) for k in ("Px", "Ax", "q", "l", "u")]
    d = DeviceBatch(b["P"], b["A"], B, device=0, **s)
    o = (torch.empty((B, b["n"]), dtype=torch.float64, device=dev),
         torch.empty((B, b["m"]), dtype=torch.float64, device=dev),
         torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.int32, device=dev))
    d.setup(*X)
    d.solve(*o)
    d.synchronize()
    assert np.array_equal(rh.x, o[0].cpu().numpy()) and np.array_equal(rh.y, o[1].cpu().numpy())
    assert np.array_equal(rh.status_val, o[2].cpu().numpy()) and np.array_equal(rh.iter, o[3].cpu().numpy())
    assert (rh.status_val == 1).all() and (rh.status_polish == 0).all()
    assert np.isfinite(rh.obj_val).all() and (rh.pri_res >= 0).all() and (rh.dua_res >= 0).all()


def test_invalid_update_reports_zero_iterations():
    """An instance whose update() makes its bounds invalid (l > u) exits before any
    ADMM iteration: status 'non convex' with NaN outputs (osqp refuses such data) and
    an iteration count of 0 -- not the previous solve's count, which the next solve's
    dispatch order (kernels.hip::k_order) would otherwise rank as a long solve."""
    import torch
    from osqp_amd import DeviceBatch
    B = 8
    b = mpc.make_batch(2, B=B, seed=5)
    s = {k: v for k, v in b["settings"].items() if k != "verbose"}
    dev = torch.device("cuda", 0)
    X = [torch.from_numpy(np.ascontiguousarray(b[k])).to(dev) for k in ("Px", "Ax", "q", "l", "u")]
    x = torch.empty((B, b["n"]), dtype=torch.float64, device=dev)
    y = torch.empty((B, b["m"]), dtype=torch.float64, device=dev)
    st = torch.empty(B, dtype=torch.int32, device=dev)
    it = torch.empty(B, dtype=torch.int32, device=dev)
    h = DeviceBatch(b["P"], b["A"], B, device=0, **s)
    h.setup(*X)
    h.solve(x, y, st, it)
    h.synchronize()
    assert (it.cpu().numpy() > 0).all()
    bad = X[3].clone()
    bad[3, 10] = X[4][3, 10] + 1.0  # lower bound above the upper one, instance 3 only
    h.update(l=bad)
    h.solve(x, y, st, it)
    h.synchronize()
    stv, itv = st.cpu().numpy(), it.cpu().numpy()
    assert stv[3] == -7 and itv[3] == 0
    assert torch.isnan(x[3]).all()
    assert (stv[np.arange(B) != 3] == 1).all() and (itv[np.arange(B) != 3] > 0).all()


def test_calls_on_different_streams_are_ordered():
    """Consecutive calls on one handle enqueued on different streams, with no
    synchronisation in between: the library orders each call after the previous one
    (api.hip::stream_enter), so the results equal a single-stream run."""
    import torch
    from osqp_amd import DeviceBatch
    B = 1024
    bx, by = mpc.make_batch(2, B=B, seed=31), mpc.make_batch(2, B=B, seed=32)
    s = {k: v for k, v in bx["settings"].items() if k != "verbose"}
    s.update(warm_start=False)
    dev = torch.device("cuda", 0)
    n, m = bx["n"], bx["m"]

    def put(b):
        return [torch.from_numpy(np.ascontiguousarray(b[k])).to(dev) for k in ("Px", "Ax", "q", "l", "u")]

    def out():
        return (torch.empty((B, n), dtype=torch.float64, device=dev), torch.empty((B, m), dtype=torch.float64, device=dev),
                torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.int32, device=dev))

    X, Y = put(bx), put(by)
    torch.cuda.synchronize()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    h = DeviceBatch(bx["P"], bx["A"], B, device=0, **s)
    o1, o2 = out(), out()
    h.setup(*X, stream=sa.cuda_stream)
    h.solve(*o1, stream=sa.cuda_stream)   # k_order rewrites the dispatch order on sa ...
    h.setup(*Y, stream=sb.cuda_stream)    # ... which this setup and solve on sb must wait for
    h.solve(*o2, stream=sb.cuda_stream)
    torch.cuda.synchronize()
    ref = DeviceBatch(bx["P"], bx["A"], B, device=0, **s)
    r1, r2 = out(), out()
    ref.setup(*X); ref.solve(*r1)
    ref.setup(*Y); ref.solve(*r2)
    ref.synchronize()
    for a, c in zip(o1 + o2, r1 + r2):
        assert torch.equal(a, c)


def test_own_stream_calls_are_ordered_without_events():
    """A call on the handle's own stream records no event (no packet between a single-stream
    caller's kernels); moving to a caller's stream records the ordering event on the own
    stream first (api.hip::stream_enter), and moving back waits for the caller stream's.
    Own -> caller -> own with no synchronisation in between equals a single-stream run.
    mpcqp_last_kernel_ms is -1 for a device solve without timing, a time with it."""
    import torch
    from osqp_amd import DeviceBatch, lib
    B = 1024
    bs = [mpc.make_batch(2, B=B, seed=41 + k) for k in range(3)]
    s = {k: v for k, v in bs[0]["settings"].items() if k != "verbose"}
    s.update(warm_start=False)
    dev = torch.device("cuda", 0)
    n, m = bs[0]["n"], bs[0]["m"]

    def put(b):
        return [torch.from_numpy(np.ascontiguousarray(b[k])).to(dev) for k in ("Px", "Ax", "q", "l", "u")]

    def out():
        return (torch.empty((B, n), dtype=torch.float64, device=dev), torch.empty((B, m), dtype=torch.float64, device=dev),
                torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.int32, device=dev))

    ins = [put(b) for b in bs]
    torch.cuda.synchronize()
    sc = torch.cuda.Stream()
    h = DeviceBatch(bs[0]["P"], bs[0]["A"], B, device=0, **s)
    o = [out() for _ in range(3)]
    h.setup_solve(*ins[0], *o[0])                          # own stream
    assert lib().mpcqp_last_kernel_ms(h._h.ptr) == -1.0    # no event pair without timing
    h.setup_solve(*ins[1], *o[1], stream=sc.cuda_stream)   # caller stream: waits for the own stream
    h.setup_solve(*ins[2], *o[2])                          # own stream again: waits for the caller's
    h.synchronize()
    torch.cuda.synchronize()
    ref = DeviceBatch(bs[0]["P"], bs[0]["A"], B, device=0, **s)
    r = [out() for _ in range(3)]
    for k in range(3):
        ref.setup_solve(*ins[k], *r[k])
    ref.synchronize()
    for a, c in zip(sum(map(list, o), []), sum(map(list, r), [])):
        assert torch.equal(a, c)
    ref.timing(True)
    ref.setup_solve(*ins[0], *r[0])
    assert lib().mpcqp_last_kernel_ms(ref._h.ptr) > 0.0
    ref.timing(False)
    # mask 2 alone: setup launches timed, solve launches not (mpcqp.h::mpcqp_timing)
    lib().mpcqp_timing(ref._h.ptr, 2)
    ref.setup(*ins[1])
    ref.solve(*r[1])
    ref.synchronize()
    kt = ref.timing_read()
    assert kt["n_setup"] == 1 and kt["setup_ms"] > 0.0 and kt["n_solve"] == 0, kt
    ref.timing(False)


@pytest.mark.parametrize("cfg,B", [(2, 512), (3, 512)])
def test_register_list_setup_is_bit_identical(monkeypatch, cfg, B):
    """kernels.hip::k_setup_r (register-resident gather lists, one column / row per
    thread) against the staged-index k_setup (MPCQP_SETUP_STAGED=1): the same Ruiz
    scaling arithmetic in the same order, so the solves that follow agree bit for bit."""
    import torch
    from osqp_amd import DeviceBatch
    b = mpc.make_batch(cfg, B=B, seed=77)
    s = {k: v for k, v in b["settings"].items() if k != "verbose"}
    dev = torch.device("cuda", 0)
    X = [torch.from_numpy(np.ascontiguousarray(b[k])).to(dev) for k in ("Px", "Ax", "q", "l", "u")]

    def run():
        h = DeviceBatch(b["P"], b["A"], B, device=0, **s)
        o = (torch.empty((B, b["n"]), dtype=torch.float64, device=dev),
             torch.empty((B, b["m"]), dtype=torch.float64, device=dev),
             torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.int32, device=dev))
        h.setup(*X)
        h.solve(*o)
        h.synchronize()
        return o

    fast = run()
    monkeypatch.setenv("MPCQP_SETUP_STAGED", "1")
    staged = run()
    for a, c in zip(fast, staged):
        assert torch.equal(a, c)


@pytest.mark.parametrize("cfg,B", [(2, 1024), (2, 40), (3, 96)])
def test_fused_setup_solve_is_bit_identical(cfg, B):
    """mpcqp_setup_solve_device (one kernel for the four- and two-wave variants:
    solve_wave.hip::k_setup_solve_w4 / _w2; setup + solve kernels otherwise) against setup_device +
    solve_device on a second handle: identical outputs, over two consecutive batches
    (the second dispatched in the order the first left behind)."""
    import torch
    from osqp_amd import DeviceBatch
    bx, by = mpc.make_batch(cfg, B=B, seed=41), mpc.make_batch(cfg, B=B, seed=42)
    s = {k: v for k, v in bx["settings"].items() if k != "verbose"}
    dev = torch.device("cuda", 0)
    n, m = bx["n"], bx["m"]

    def put(b):
        return [torch.from_numpy(np.ascontiguousarray(b[k])).to(dev) for k in ("Px", "Ax", "q", "l", "u")]

    def out():
        return (torch.empty((B, n), dtype=torch.float64, device=dev), torch.empty((B, m), dtype=torch.float64, device=dev),
                torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.int32, device=dev))

    X, Y = put(bx), put(by)
    fused, sep = DeviceBatch(bx["P"], bx["A"], B, device=0, **s), DeviceBatch(bx["P"], bx["A"], B, device=0, **s)
    for D in (X, Y):
        of, os_ = out(), out()
        fused.setup_solve(*D, *of)
        sep.setup(*D)
        sep.solve(*os_)
        torch.cuda.synchronize()
        for a, c in zip(of, os_):
            assert torch.equal(a, c)
    assert (of[2] == 1).all()


@pytest.mark.parametrize("N", [50, 100])
def test_slack_script_default_horizon(N):
    """The slack script as it ships (vehicle_lateral_mpc_slack_increment.py:14, N = 100;
    and N = 50): one instance, 37 / 19 factor blocks -- past the register-resident
    kernels, so the generic workspace-tile path (variants 4-6) or the long-horizon
    kernel runs it.  Same status, iterations and du_0 as the oracle."""
    x0 = np.array([0.0, 0.0, 5 * mpc.DEG, 3.0, 0.0])
    P, q, A, l, u = mpc.slack_qp(N, x0)
    nx = 5
    _cmp_single(P, q, A, l, u, dict(warm_start=True), slice((N + 1) * nx, (N + 1) * nx + N))


def _random_banded_batch(B, n, m, band, seed):
    """Random strictly convex QPs with a banded (non-MPC) sparsity pattern shared by the
    batch: P = L L' + I restricted to the band, A rows of <= 2 band + 1 nonzeros, boxes
    mixed with equality and one-sided rows.  Exercises the plan's level-set blocking on
    patterns the reference's builders never produce."""
    import scipy.sparse as sp
    rng = np.random.default_rng(seed)
    ii, jj = [], []
    for i in range(n):
        for j in range(max(0, i - band), min(n, i + band + 1)):
            ii.append(i); jj.append(j)
    Pp = sp.csc_matrix((np.ones(len(ii)), (ii, jj)), shape=(n, n))
    Pp = sp.triu(Pp).tocsc()
    ai, aj = [], []
    for r in range(m):
        c = rng.integers(0, n)
        for j in range(max(0, c - band), min(n, c + band + 1)):
            if rng.random() < 0.6 or j == c:
                ai.append(r); aj.append(j)
    Ap = sp.csc_matrix((np.ones(len(ai)), (ai, aj)), shape=(m, n))
    Ap.sort_indices(); Pp.sort_indices()
    Px = np.empty((B, Pp.nnz)); Ax = rng.normal(size=(B, Ap.nnz))
    pr = Pp.indices  # CSC storage order
    pc = np.repeat(np.arange(n), np.diff(Pp.indptr))
    for k in range(B):
        M = rng.normal(size=(n, n)) * 0.3
        Md = sp.csc_matrix(np.where(np.abs(np.subtract.outer(np.arange(n), np.arange(n))) <= band, M @ M.T, 0.0)
                           + (2.0 * band + 2.0) * np.eye(n))  # diagonally dominant: SPD
        Px[k] = np.asarray(Md[pr, pc]).ravel()
    q = rng.normal(size=(B, n))
    l = rng.uniform(-2, -0.1, size=(B, m)); u = rng.uniform(0.1, 2, size=(B, m))
    kind = rng.integers(0, 4, size=m)
    l[:, kind == 1] = u[:, kind == 1]         # equality rows
    l[:, kind == 2] = -np.inf                 # one-sided
    u[:, kind == 3] = np.inf
    return dict(P=Pp, A=Ap, Px=Px, Ax=Ax, q=q, l=l, u=u, u_block=slice(0, n))


@pytest.mark.parametrize("n,m,band,seed", [(60, 40, 2, 1), (150, 90, 3, 2), (300, 200, 1, 3)])
def test_random_banded_qps(n, m, band, seed):
    """Non-MPC sparsity (random banded P and A) through the generic kernels (variants 6
    and 11 here).  The batches mix solved, primal-infeasible, max-iteration and inaccurate
    instances and need up to 1,050 iterations -- long ADMM runs on far worse conditioned
    systems than the MPC layouts, where rounding-level differences between linear solvers
    grow.  tools/diag_random.py (profiles/r3_diag_random_banded.txt) puts three solvers side
    by side: the statuses agree on all 288 instances; the iteration counts on all but two,
    both in the first batch -- instance 55 (device 975, oracle 1,050, the dense numpy
    restatement 1,050) and instance 85 (500 / 525 / 425: the two CPU solvers, equal in exact
    arithmetic, disagree as well).  The reduced matrix P + sigma I + A' rho A the device
    factors is 15-18x worse conditioned there than the quasi-definite KKT matrix OSQP
    factors (about 5e2 vs 3e1; not the square), and those two instances are the batch's
    longest solves.  Bar: statuses equal for >= 99 %, iteration counts for >= 95 %; where
    both agree, x within 5e-3 relative (eps-level: the first batch's worst such instance is
    1.5e-3 apart after 525 identical-count iterations) with a median below 1e-6; and every
    instance the device reports solved meets the termination test it claims, recomputed on
    the host from the returned (x, y) in unscaled form: dist(Ax, [l, u]) <= eps_abs +
    eps_rel ||Ax|| and ||Px + q + A'y|| <= eps_abs + eps_rel max(||Px||, ||A'y||, ||q||)
    (inf-norms; z is within eps_prim of Ax, so the box distance can only be smaller than
    OSQP's residual)."""
    b = _random_banded_batch(96, n, m, band, seed)
    s = dict(warm_start=False, polish=False)
    bo = pyoracle.solve_batch(b["P"], b["A"], b["Px"], b["q"], b["Ax"], b["l"], b["u"], nthreads=16, **s)
    bg = OSQPBatch()
    bg.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
    rg = bg.solve()
    assert np.mean(rg.status_val == bo.status_val) >= 0.99
    assert np.mean(rg.iter == bo.iter) >= 0.95
    same = (rg.iter == bo.iter) & (rg.status_val == bo.status_val) & np.isfinite(bo.x).all(axis=1)
    dx = np.abs(rg.x - bo.x).max(axis=1) / np.maximum(1.0, np.abs(bo.x).max(axis=1))
    assert np.all(dx[same] < 5e-3), dx[same].max()
    assert np.median(dx[same]) < 1e-6
    P, A = b["P"].copy(), b["A"].copy()
    for k in np.flatnonzero(rg.status_val == 1):
        P.data, A.data = b["Px"][k], b["Ax"][k]
        x, y = rg.x[k], rg.y[k]
        ax = A @ x
        px = P @ x + P.T @ x - P.diagonal() * x
        aty = A.T @ y
        prim = np.max(np.maximum(0.0, np.maximum(ax - b["u"][k], b["l"][k] - ax)))
        dual = np.abs(px + b["q"][k] + aty).max()
        assert prim <= (1e-3 + 1e-3 * np.abs(ax).max()) * 1.01, (k, prim)
        assert dual <= (1e-3 + 1e-3 * max(np.abs(px).max(), np.abs(aty).max(), np.abs(b["q"][k]).max())) * (1 + 1e-9), (k, dual)


@pytest.mark.parametrize("eps", [1e-3, 1e-9])
def test_osqp_demo_known_answer(eps):
    """OSQP's documented demo problem (tests/test_oracle.py::osqp_demo_problem): the
    device matches the oracle (status, iterations, x) and the closed-form optimum."""
    from test_oracle import osqp_demo_problem
    P, q, A, l, u, xs, ys, obj = osqp_demo_problem()
    ro, rg = _cmp_single(P, q, A, l, u, dict(eps_abs=eps, eps_rel=eps), slice(0, 2))
    tol = 5e-3 if eps > 1e-6 else 1e-7
    assert np.abs(rg.x - xs).max() < tol
    assert np.abs(rg.y - ys).max() < 10 * tol


@pytest.mark.parametrize("cfg,B", [(2, 1024), (3, 512)])
def test_repeat_solves_are_bitwise_identical(cfg, B):
    """The same batch solved on three fresh handles gives bitwise identical outputs: no
    result may depend on the timing of the waves inside a workgroup.  (A missing barrier
    between the y park and the factorisation's scratch made one instance in ~4 runs of
    cfg 2 drift by 1e-5 in the four-wave kernel before it was fixed.)"""
    b = mpc.make_batch(cfg, B=B)
    s = dict(warm_start=True)
    outs = []
    for _ in range(3):
        bg = OSQPBatch()
        bg.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
        outs.append(bg.solve())
    for r in outs[1:]:
        assert np.array_equal(r.x, outs[0].x) and np.array_equal(r.y, outs[0].y)
        assert np.array_equal(r.iter, outs[0].iter)


@pytest.mark.parametrize("B", [512, 1000])
def test_slack_elimination_matches_full_system(monkeypatch, B):
    """The slack layout runs the four-wave kernel on its reduced system (plan.h Plan::eown:
    105 slack columns eliminated by a scalar Schur complement, 125 variables in 4 blocks);
    MPCQP_ELIM=0 runs the full 230-variable system (8 blocks, the 256-thread register-sweep
    kernel).  Both must match the oracle and each other: same statuses, iteration counts
    for >= 99 % of the instances, and u within the north-star 1e-4."""
    b = mpc.make_batch(3, B=B, seed=13)
    s = dict(warm_start=True)
    bg = OSQPBatch()
    bg.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
    info = bg.plan_info()
    assert (info["nb"], info["n_eliminated"], info["variant"]) == (4, 105, 17)
    rg = bg.solve()
    monkeypatch.setenv("MPCQP_ELIM", "0")
    bf = OSQPBatch()
    bf.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
    assert bf.plan_info()["n_eliminated"] == 0 and bf.plan_info()["nb"] == 8
    rf = bf.solve()
    assert (rg.status_val == rf.status_val).all()
    same = rg.iter == rf.iter
    assert same.mean() >= 0.99
    du = np.abs(rg.x[:, b["u_block"]] - rf.x[:, b["u_block"]]).max(axis=1)
    assert np.all(du[same] < U_TOL), du.max()
    # slack values (the eliminated columns) agree too
    sl = slice(125, 230)
    assert np.all(np.abs(rg.x[same][:, sl] - rf.x[same][:, sl]).max(axis=1) < 1e-4)


@pytest.mark.parametrize("cfg,nb,ne,variant", [(2, 4, 0, 17), (3, 4, 105, 17), (5, 17, 0, 12)])
def test_plan_and_kernel_per_config(cfg, nb, ne, variant):
    """The plan and solve kernel each BASELINE workload runs with (guards against a plan
    change moving a config to another kernel: cfg 5 on a greedily packed plan -- 16 blocks,
    15 coupling rows -- ran 2x slower in the long-horizon kernel)."""
    b = mpc.make_batch(cfg, B=4, seed=1)
    bg = OSQPBatch()
    bg.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"],
             **{k: v for k, v in b["settings"].items() if k != "verbose"})
    info = bg.plan_info()
    assert (info["nb"], info["n_eliminated"], info["variant"]) == (nb, ne, variant)


@pytest.mark.parametrize("cfg,B,warm", [(2, 64, False), (2, 64, True), (3, 48, True), (5, 12, False)])
def test_matrix_updates_match_oracle(cfg, B, warm):
    """update(Px=, Ax=, Ax_idx=) -- mpcqp_update_matrices_batch, OSQP 0.6 osqp_update_P_A:
    unscale, new values, rescale, refactor at the next solve, iterates kept -- on cfg 2 (the
    four-wave kernel), the slack layout (its eliminated-column plan) and cfg 5 (the long-horizon
    kernel, the staged setup): solved, then every P value scaled by 1.5 and solved, then a third of A's values
    changed by index (with a repeated index) and solved, each against the oracle doing the
    same calls."""
    b = mpc.make_batch(cfg, B=B, seed=9)
    s = dict(warm_start=warm)
    P, A = b["P"], b["A"]
    dev = OSQPBatch()
    dev.setup(P, b["q"], A, b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
    orc = []
    for k in range(b["Px"].shape[0]):
        o = pyoracle.OSQP()
        Pk, Ak = P.copy(), A.copy()
        Pk.data, Ak.data = b["Px"][k].copy(), b["Ax"][k].copy()
        o.setup(Pk, b["q"][k], Ak, b["l"][k], b["u"][k], **s)
        orc.append(o)
    rng = np.random.default_rng(3)
    idx = np.concatenate([np.arange(0, A.nnz, 3), [0]])
    for step in range(3):
        if step == 1:
            Pn = b["Px"] * 1.5
            dev.update(Px=Pn)
            for k, o in enumerate(orc):
                o.update(Px=Pn[k])
        elif step == 2:
            spread = 0.01 if cfg == 5 else 0.1  # (cfg 5: +-10 % makes some solves ill-conditioned, 4000 iterations)
            An = b["Ax"][:, idx] * rng.uniform(1 - spread, 1 + spread, (b["Ax"].shape[0], idx.size))
            dev.update(Ax=An, Ax_idx=idx)
            for k, o in enumerate(orc):
                o.update(Ax=An[k], Ax_idx=idx)
        rd = dev.solve()
        ro = [o.solve() for o in orc]
        st = np.array([r.info.status_val for r in ro])
        it = np.array([r.info.iter for r in ro])
        # (cfg 5: solves of up to ~2000 iterations; at most one instance a check interval apart,
        # the linear-solver difference of DESIGN.md §3)
        bar = 1.0 - 1.0 / B if cfg == 5 else 0.99
        assert np.mean(rd.status_val == st) >= bar, step
        assert np.mean(rd.iter == it) >= bar, step
        same = (rd.iter == it) & (st == 1)
        assert same.sum() >= 0.9 * len(ro) - 1, step
        du = np.array([np.abs(rd.x[k, b["u_block"]] - ro[k].x[b["u_block"]]).max() for k in range(len(ro))])
        assert np.all(du[same] < U_TOL), (step, du[same].max())


def test_shim_matrix_update_demo():
    """osqp.OSQP().update(Px=, Px_idx=, Ax=, Ax_idx=) through the shim on the osqp
    documentation's demo problem and its update_P_A example, with an index update after
    it: the same iteration counts as the oracle and x to 1e-9."""
    import scipy.sparse as sps
    P = sps.csc_matrix(np.array([[4.0, 1.0], [1.0, 2.0]]))
    A = sps.csc_matrix(np.array([[1.0, 1.0], [1.0, 0.0], [0.0, 1.0]]))
    q, l, u = np.array([1.0, 1.0]), np.array([1.0, 0.0, 0.0]), np.array([1.0, 0.7, 0.7])
    s = dict(eps_abs=1e-6, eps_rel=1e-6, verbose=False)
    g, o = OSQP(), pyoracle.OSQP()
    g.setup(P, q, A, l, u, **s)
    o.setup(P, q, A, l, u, **s)
    calls = [dict(),
             dict(Px=np.array([5.0, 1.5, 1.0]), Ax=np.array([1.2, 1.5, 1.1, 0.8])),
             dict(Px=np.array([3.0]), Px_idx=np.array([0]), Ax=np.array([0.9, 1.0]), Ax_idx=np.array([2, 2]))]
    for c in calls:
        if c:
            g.update(**c)
            o.update(**c)
        rg, ro = g.solve(), o.solve()
        assert rg.info.status == ro.info.status == "solved"
        assert rg.info.iter == ro.info.iter
        assert np.abs(rg.x - ro.x).max() < 1e-9


def test_matrix_update_keeps_the_pattern():
    """An entry that is zero in every instance at setup is not in the device's pattern:
    setting it nonzero is refused (run setup again), keeping it zero is fine."""
    import scipy.sparse as sps
    # triu(P) with an explicit zero at (0, 1): in osqp's pattern, dropped from the device's
    P = sps.csc_matrix((np.array([4.0, 0.0, 2.0]), np.array([0, 0, 1]), np.array([0, 1, 3])), shape=(2, 2))
    A = sps.csc_matrix(np.array([[1.0, 1.0], [1.0, 0.0], [0.0, 1.0]]))
    q, l, u = np.array([1.0, 1.0]), np.array([1.0, 0.0, 0.0]), np.array([1.0, 0.7, 0.7])
    g = OSQP()
    g.setup(P, q, A, l, u, verbose=False)
    g.solve()
    with pytest.raises(ValueError):
        g.update(Px=np.array([4.0, 1.0, 2.0]))
    g.update(Px=np.array([5.0, 0.0, 2.0]))
    assert g.solve().info.status == "solved"


def test_nonconvex_setup_raises_like_osqp():
    """osqp_setup refuses a problem whose KKT matrix is not quasi-definite (a non-convex P):
    osqp-python raises ValueError at setup, and so do the shim and OSQPBatch
    (api.hip::check_convex, one factor-only launch) -- for a single QP, for one bad instance
    in a cfg-2 batch (the four-wave kernel's factor-only instantiation), and for a matrix
    update that makes P non-convex.  The oracle rejects the same problems."""
    import scipy.sparse as sps
    P = sps.csc_matrix(np.array([[-1.0, 0.0], [0.0, 1.0]]))
    A = sps.csc_matrix(np.array([[1.0, 1.0]]))
    q, l, u = np.zeros(2), np.array([-1.0]), np.array([1.0])
    with pytest.raises(ValueError):
        pyoracle.OSQP().setup(P, q, A, l, u)
    with pytest.raises(ValueError, match="not convex"):
        OSQP().setup(P, q, A, l, u, verbose=False)
    b = mpc.make_batch(2, B=64, seed=12)
    s = {k: v for k, v in b["settings"].items() if k != "verbose"}
    Px = b["Px"].copy()
    Px[37] *= -1.0
    h = OSQPBatch()
    with pytest.raises(ValueError, match="instance 37"):
        h.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=Px, Ax=b["Ax"], **s)
    h.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
    assert h.plan_info()["variant"] == 17
    assert (h.solve().status_val == 1).all()
    with pytest.raises(ValueError, match="instance 37"):
        h.update(Px=Px)


def test_nonconvex_eliminated_slack_raises_like_osqp():
    """The slack layout's plan eliminates the slack columns (plan.h Plan::eown): their pivot
    K_jj = P_jj + sigma + rho a^2 never enters the reduced block factor, so a negative slack
    weight is caught by factorize_w4's own check of K_jj (the reduced blocks alone would still
    factor: subtracting a negative Schur term raises the parent's diagonal).  A live slack's
    weight -10 (the e_y slack of stage 3, P column 143): the oracle rejects it, and so must
    setup() and update(Px=) -- ValueError naming the instance."""
    b = mpc.make_batch(3, B=48, seed=12)
    s = {k: v for k, v in b["settings"].items() if k != "verbose"}
    P = b["P"]
    pos = P.indptr[143]
    assert P.indices[pos] == 143 and P.indptr[144] - pos == 1
    Px = b["Px"].copy()
    Px[5, pos] = -10.0
    Pk = P.copy()
    Pk.data = Px[5].copy()
    with pytest.raises(ValueError):
        pyoracle.OSQP().setup(Pk, b["q"][5], b["A"], b["l"][5], b["u"][5], verbose=False)
    h = OSQPBatch()
    with pytest.raises(ValueError, match="instance 5"):
        h.setup(P, b["q"], b["A"], b["l"], b["u"], Px=Px, Ax=b["Ax"], **s)
    h.setup(P, b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
    assert h.plan_info()["n_eliminated"] > 0
    with pytest.raises(ValueError, match="instance 5"):
        h.update(Px=Px)
    # After a solve the KKT matrix is refactored with the rho vector the solve adapted to
    # (orc_update_P_A, OSQP 0.6 osqp_update_P_A): instance 5's rho grew (200 iterations,
    # one rho update), so sigma + rho a^2 now outweighs a weight of -10 and OSQP accepts the
    # update -- and so must the device; a weight of -1000 is refused by both.
    for w, refused in ((-10.0, False), (-1000.0, True)):
        Px[5, pos] = w
        Pk.data = Px[5].copy()
        Ak = b["A"].copy()
        Ak.data = b["Ax"][5].copy()
        Pg = P.copy()
        Pg.data = b["Px"][5].copy()
        o = pyoracle.OSQP()
        o.setup(Pg, b["q"][5], Ak, b["l"][5], b["u"][5], **s)
        o.solve()
        h = OSQPBatch()
        h.setup(P, b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
        assert (h.solve().status_val == 1).all()
        if refused:
            with pytest.raises(ValueError):
                o.update(Px=Pk.data)
            with pytest.raises(ValueError, match="instance 5"):
                h.update(Px=Px)
        else:
            o.update(Px=Pk.data)
            h.update(Px=Px)


@pytest.mark.parametrize("cfg,B", [(2, 64), (3, 48), (5, 12)])
def test_update_settings_match_oracle(cfg, B):
    """update_settings (mpcqp_update_settings, osqp_update_settings / osqp_update_rho): on a
    cfg-2 batch solved once, then tighter tolerances, a new rho (refactored, row classes
    kept), alpha, max_iter and check interval, solved warm; then warm starting off, solved
    cold -- each against the oracle doing the same calls.  Settings OSQP fixes at setup are
    refused by both."""
    b = mpc.make_batch(cfg, B=B, seed=21)
    s = dict(warm_start=True)
    P, A = b["P"], b["A"]
    dev = OSQPBatch()
    dev.setup(P, b["q"], A, b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
    orc = []
    for k in range(b["Px"].shape[0]):
        o = pyoracle.OSQP()
        Pk, Ak = P.copy(), A.copy()
        Pk.data, Ak.data = b["Px"][k].copy(), b["Ax"][k].copy()
        o.setup(Pk, b["q"][k], Ak, b["l"][k], b["u"][k], **s)
        orc.append(o)
    # (the third call passes no rho: each instance keeps the rho its previous solve adapted to,
    # on the device and in the oracle, as osqp-python calls update_rho only when rho is given)
    for step, kw in enumerate([{}, dict(eps_abs=1e-4, eps_rel=1e-4, rho=0.5, alpha=1.4, max_iter=3000,
                                        check_termination=10),
                               dict(warm_start=False)]):
        if kw:
            dev.update_settings(**kw)
            for o in orc:
                o.update_settings(**kw)
        rd = dev.solve()
        ro = [o.solve() for o in orc]
        st = np.array([r.info.status_val for r in ro])
        it = np.array([r.info.iter for r in ro])
        bar = 1.0 - 1.0 / B if cfg == 5 else 0.99  # (as in test_matrix_updates_match_oracle)
        assert np.mean(rd.status_val == st) >= bar, step
        assert np.mean(rd.iter == it) >= bar, step
        same = rd.iter == it
        du = np.array([np.abs(rd.x[k, b["u_block"]] - ro[k].x[b["u_block"]]).max() for k in range(len(ro))])
        assert np.all(du[same] < U_TOL), (step, du[same].max())
        if step == 1:  # every 10 iterations now
            assert np.all(rd.iter % 10 == 0)
    with pytest.raises(ValueError):
        dev.update_settings(sigma=1e-5)
    with pytest.raises(ValueError):
        orc[0].update_settings(sigma=1e-5)


def test_update_settings_polish_on_eliminated_plan(golden):
    """update_settings(polish=True) on a slack-layout handle set up without polish, whose plan
    eliminated the 105 slack columns (api.hip::replan_plain moves it onto the plain plan,
    state kept): the warm re-solve after it matches the oracle doing the same calls -- the
    reference's own slack QP through the shim, and a cfg-3 batch (status, iterations, polish
    decision, x)."""
    g = golden("slack_n20.npz")
    P, A, q, l, u = g["P"], g["A"], g["q"], g["l"], g["u"]
    d, o = OSQP(), pyoracle.OSQP()
    d.setup(P, q, A, l, u, warm_start=True, verbose=False)
    o.setup(P, q, A, l, u, warm_start=True)
    d.solve(); o.solve()
    d.update_settings(polish=True)
    o.update_settings(polish=True)
    # the reference's own update of step 401 (bound regime 1; the script's update, :237)
    q2, l2, u2 = g["upd_q"][1], g["upd_l"][1], g["upd_u"][1]
    d.update(q=q2, l=l2, u=u2); o.update(q=q2, l=l2, u=u2)
    rd, ro = d.solve(), o.solve()
    assert rd.info.status == ro.info.status and rd.info.iter == ro.info.iter
    assert rd.info.status_polish == ro.info.status_polish
    tol = 1e-8 if ro.info.status_polish == 1 else 1e-6
    assert np.abs(rd.x - ro.x).max() < tol * max(1.0, np.abs(ro.x).max())

    b = mpc.make_batch(3, B=48, seed=31)
    s = dict(warm_start=True)
    dev = OSQPBatch()
    dev.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
    assert dev.plan_info()["n_eliminated"] == 105
    r0 = dev.solve()
    orc = []
    for k in range(b["Px"].shape[0]):
        ok = pyoracle.OSQP()
        Pk, Ak = b["P"].copy(), b["A"].copy()
        Pk.data, Ak.data = b["Px"][k].copy(), b["Ax"][k].copy()
        ok.setup(Pk, b["q"][k], Ak, b["l"][k], b["u"][k], **s)
        ok.solve()
        ok.update_settings(polish=True)
        orc.append(ok)
    dev.update_settings(polish=True)
    info = dev.plan_info()
    assert info["n_eliminated"] == 0 and info["plan_choice"] == 0
    lb, ub = b["l"].copy(), b["u"].copy()
    lb[:, :5] = ub[:, :5] = b["l"][:, :5] * 0.95
    dev.update(l=lb, u=ub)
    rd = dev.solve()
    ros = []
    for k, ok in enumerate(orc):
        ok.update(l=lb[k], u=ub[k])
        ros.append(ok.solve())
    it = np.array([r.info.iter for r in ros])
    ps = np.array([r.info.status_polish for r in ros])
    assert (rd.status_val == 1).all() and (r0.status_val == 1).all()
    assert (rd.iter == it).mean() >= 0.97, (rd.iter, it)
    same = rd.iter == it
    assert (rd.status_polish[same] == ps[same]).all()
    xo = np.stack([r.x for r in ros])
    assert np.abs(rd.x[same] - xo[same]).max() < 1e-6 * max(1.0, np.abs(xo).max())


def test_replan_matches_a_handle_set_up_on_the_plain_plan(monkeypatch):
    """Device against device: a cfg-3 handle set up on the eliminated plan, solved,
    then re-planned by update_settings(polish=True) (api.hip::replan_plain) and warm-started,
    against a handle set up on the plain plan directly (polish on) from the same (x, y).  With
    adaptive rho off both carry rho = 0.1, the same scaling and z = Ax, so every per-column and
    per-row array the re-plan permutes must land where the plain plan's setup puts it: the next
    solve agrees on every instance -- status, iterations, polish decision -- and x, y to rounding."""
    b = mpc.make_batch(3, B=96, seed=41)
    s = dict(warm_start=True, adaptive_rho=False, max_iter=400)
    a = OSQPBatch()
    a.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
    assert a.plan_info()["n_eliminated"] == 105
    r0 = a.solve()
    x0, y0 = r0.x.copy(), r0.y.copy()
    a.update_settings(polish=True)
    assert a.plan_info()["n_eliminated"] == 0 and a.plan_info()["plan_choice"] == 0
    c = OSQPBatch()
    c.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **dict(s, polish=True))
    assert c.plan_info()["n_eliminated"] == 0 and c.plan_info()["plan_choice"] == 0
    lb, ub = b["l"].copy(), b["u"].copy()
    lb[:, :5] = ub[:, :5] = b["l"][:, :5] * 0.97
    for h in (a, c):
        h.warm_start(x=x0, y=y0)
        h.update(l=lb, u=ub)
    ra, rc = a.solve(), c.solve()
    assert (ra.status_val == rc.status_val).all()
    assert (ra.iter == rc.iter).all(), (ra.iter, rc.iter)
    assert (ra.status_polish == rc.status_polish).all()
    assert np.abs(ra.x - rc.x).max() <= 1e-12 * max(1.0, np.abs(rc.x).max())
    assert np.abs(ra.y - rc.y).max() <= 1e-12 * max(1.0, np.abs(rc.y).max())


@pytest.mark.parametrize("cfg,B", [(2, 256), (3, 128)])
def test_four_wave_factor_reuse_is_exact(monkeypatch, cfg, B):
    """The stand-alone four-wave solve kernel (k_solve_w4, the host API's solve) starts from
    setup()'s convexity factor -- the factor-only launch leaves its S_k^{-1} tiles in the
    workspace -- instead of factoring again; the fused setup + solve kernel is untouched.  A handle
    that reuses it and one that refactors (MPCQP_FACTOR_REUSE=0) agree bit for bit through solve,
    update(q), solve, update(l, u) moving row classes, solve (cfg 2 plain, cfg 3 eliminated plan)."""
    b = mpc.make_batch(cfg, B=B, seed=19)
    s = dict(warm_start=True)
    hs = []
    for reuse in ("1", "0"):
        monkeypatch.setenv("MPCQP_FACTOR_REUSE", reuse)
        h = OSQPBatch()
        h.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
        hs.append(h)
    monkeypatch.delenv("MPCQP_FACTOR_REUSE")
    l3, u3 = b["l"].copy(), b["u"].copy()
    fin = np.isfinite(l3[0]) & np.isfinite(u3[0]) & (u3[0] - l3[0] > 1e-3)
    rows = np.flatnonzero(fin)[-4:]
    mid = 0.5 * (l3[:, rows] + u3[:, rows])
    l3[:, rows] = mid
    u3[:, rows] = mid
    for step, kw in enumerate([dict(), dict(q=b["q"] * 1.01), dict(l=l3, u=u3)]):
        for h in hs:
            if kw:
                h.update(**kw)
        r1, r0 = hs[0].solve(), hs[1].solve()
        assert np.array_equal(r1.status_val, r0.status_val) and np.array_equal(r1.iter, r0.iter), step
        assert np.array_equal(r1.x, r0.x) and np.array_equal(r1.y, r0.y), step
        if step == 0:
            assert (r1.status_val == 1).all()


def test_handles_share_a_cached_plan_through_a_replan():
    """Handles of one sparsity pattern share the plan cache's read-only plan (api.hip::cached_plan
    hands out a shared pointer, no copy).  Re-planning one of them (update_settings(polish=True):
    replan_plain) must leave the others on the shared plan, solving as before: a second handle of
    the same pattern keeps its eliminated plan and its results are bit-identical to a third,
    untouched one; and a fourth handle set up after the re-plan still gets the eliminated plan."""
    b = mpc.make_batch(3, B=64, seed=43)
    s = dict(warm_start=True)
    hs = []
    for _ in range(3):
        h = OSQPBatch()
        h.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
        assert h.plan_info()["n_eliminated"] == 105
        hs.append(h)
    hs[0].solve()
    hs[0].update_settings(polish=True)
    assert hs[0].plan_info()["n_eliminated"] == 0
    r1, r2 = hs[1].solve(), hs[2].solve()
    assert hs[1].plan_info()["n_eliminated"] == 105 and hs[2].plan_info()["n_eliminated"] == 105
    assert np.array_equal(r1.x, r2.x) and np.array_equal(r1.iter, r2.iter)
    assert (r1.status_val == 1).all()
    h4 = OSQPBatch()
    h4.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
    assert h4.plan_info()["n_eliminated"] == 105
    r4 = h4.solve()
    assert np.array_equal(r4.x, r1.x)
    ra = hs[0].solve()
    assert (ra.status_val == 1).all()


def test_shim_update_settings_polish_demo():
    """osqp.OSQP().update_settings(polish=True, eps_abs=, eps_rel=) through the shim on the
    osqp documentation's demo problem: polished like the oracle, the closed-form optimum."""
    import scipy.sparse as sps
    P = sps.csc_matrix(np.array([[4.0, 1.0], [1.0, 2.0]]))
    A = sps.csc_matrix(np.array([[1.0, 1.0], [1.0, 0.0], [0.0, 1.0]]))
    q, l, u = np.array([1.0, 1.0]), np.array([1.0, 0.0, 0.0]), np.array([1.0, 0.7, 0.7])
    g, o = OSQP(), pyoracle.OSQP()
    g.setup(P, q, A, l, u, verbose=False)
    o.setup(P, q, A, l, u)
    g.solve(); o.solve()
    g.update_settings(polish=True, eps_abs=1e-4, eps_rel=1e-4)
    o.update_settings(polish=True, eps_abs=1e-4, eps_rel=1e-4)
    rg, ro = g.solve(), o.solve()
    assert rg.info.iter == ro.info.iter and rg.info.status_polish == ro.info.status_polish == 1
    assert np.abs(rg.x - np.array([0.3, 0.7])).max() < 1e-9
    assert np.abs(rg.x - ro.x).max() < 1e-12


def test_long_horizon_factor_reuse_is_exact(monkeypatch):
    """The long-horizon kernel starts a solve from the workspace factor when it is the current
    one (KParams::ffresh: set by setup()'s convexity check and by every solve, cleared by a
    setup, by an update that moves a row between the equality / inequality / loose classes, by
    a rho from update_settings and by polish).  A cfg-5 handle that reuses it and one that
    refactors at every solve (MPCQP_FACTOR_REUSE=0) go through the same calls -- solve, update
    of q, update of l / u that turns rows into equalities (classes move), update_settings(rho),
    update of q again -- and agree bit for bit; both against the oracle doing the same."""
    b = mpc.make_batch(5, B=6, seed=17)
    s = dict(warm_start=True, polish=False)
    P, A = b["P"], b["A"]
    handles = []
    for reuse in ("1", "0"):
        monkeypatch.setenv("MPCQP_FACTOR_REUSE", reuse)
        h = OSQPBatch()
        h.setup(P, b["q"], A, b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
        handles.append(h)
    monkeypatch.delenv("MPCQP_FACTOR_REUSE")
    orc = []
    for k in range(b["Px"].shape[0]):
        o = pyoracle.OSQP()
        Pk, Ak = P.copy(), A.copy()
        Pk.data, Ak.data = b["Px"][k].copy(), b["Ax"][k].copy()
        o.setup(Pk, b["q"][k], Ak, b["l"][k], b["u"][k], **s)
        orc.append(o)
    q2 = b["q"] * 1.01
    l3, u3 = b["l"].copy(), b["u"].copy()
    fin = np.isfinite(l3[0]) & np.isfinite(u3[0]) & (u3[0] - l3[0] > 1e-3)
    rows = np.flatnonzero(fin)[-6:]  # inequality rows made equalities: their class moves
    mid = 0.5 * (l3[:, rows] + u3[:, rows])
    l3[:, rows] = mid
    u3[:, rows] = mid
    calls = [dict(), dict(q=q2), dict(l=l3, u=u3), dict(rho=0.3), dict(q=b["q"])]
    for step, kw in enumerate(calls):
        for h in handles:
            if "rho" in kw:
                h.update_settings(**kw)
            elif kw:
                h.update(**kw)
        for k, o in enumerate(orc):
            if "rho" in kw:
                o.update_settings(**kw)
            elif kw:
                o.update(**{n: v[k] for n, v in kw.items()})
        r1, r0 = handles[0].solve(), handles[1].solve()
        assert np.array_equal(r1.iter, r0.iter) and np.array_equal(r1.status_val, r0.status_val), step
        assert np.array_equal(r1.x, r0.x) and np.array_equal(r1.y, r0.y), step
        ro = [o.solve() for o in orc]
        it = np.array([r.info.iter for r in ro])
        assert np.mean(r1.iter == it) >= 5 / 6, (step, r1.iter, it)
        same = r1.iter == it
        du = np.array([np.abs(r1.x[k, b["u_block"]] - ro[k].x[b["u_block"]]).max() for k in range(len(ro))])
        assert np.all(du[same] < U_TOL), (step, du[same].max())


@pytest.mark.gpu
def test_dispatch_history_moves_no_result(monkeypatch):
    """The dispatch order with history (kernels.hip::k_order, KParams::pred / odecay: the default
    7/8 decay against MPCQP_ORDER_DECAY=0, the previous count alone) only moves instances
    between workgroup slots: a cfg-5 batch larger than the resident slots, solved four times
    with moving bounds (the order changes between solves), agrees bit for bit."""
    import torch
    from osqp_amd import DeviceBatch, _drop_common_zeros
    B = 1024
    b = mpc.make_batch(5, B=B, seed=29)
    P, Px = _drop_common_zeros(b["P"], b["Px"])
    A, Ax = _drop_common_zeros(b["A"], b["Ax"])
    s = {k: v for k, v in b["settings"].items() if k != "verbose"}
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    dPx, dAx, dq = t(Px), t(Ax), t(b["q"])
    rng = np.random.default_rng(3)
    bounds = []
    for k in range(4):
        l, u = b["l"].copy(), b["u"].copy()
        eq = np.isfinite(l) & np.isfinite(u) & (l == u)
        sh = rng.normal(scale=0.01, size=l.shape) * eq
        bounds.append((t(l + sh), t(u + sh)))
    torch.cuda.synchronize()
    hs = []
    for dec in ("7", "0"):
        monkeypatch.setenv("MPCQP_ORDER_DECAY", dec)
        hs.append(DeviceBatch(P, A, B, device=0, **s))
    monkeypatch.delenv("MPCQP_ORDER_DECAY")
    for l, u in bounds:
        outs = []
        for h in hs:
            o = (torch.empty((B, b["n"]), dtype=torch.float64, device=dev),
                 torch.empty((B, b["m"]), dtype=torch.float64, device=dev),
                 torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.int32, device=dev))
            h.setup(dPx, dAx, dq, l, u)
            h.solve(*o)
            h.synchronize()
            outs.append([v.cpu().numpy() for v in o])
        for a, c in zip(*outs):
            assert np.array_equal(a.view(np.int64) if a.dtype == np.float64 else a,
                                  c.view(np.int64) if c.dtype == np.float64 else c)
        assert (outs[0][2] == 1).mean() > 0.99


@pytest.mark.gpu
def test_long_horizon_lds_chain_is_exact(monkeypatch):
    """The long-horizon factorisation's chain on LDS copies of its tiles (round 6,
    solve_big.hip::factorize2s_lds_chain) against the workspace form (MPCQP_LDS_CHAIN=0): the
    same sums on the same values, so cfg-5 handles of either form agree bit for bit through a
    cold solve (setup()'s convexity factor reused), update(q) and update_settings(rho) (a
    refactorisation at the new rho) -- and every instance is solved."""
    b = mpc.make_batch(5, B=16, seed=23)
    s = dict(warm_start=True, polish=False)
    handles = []
    for on in ("1", "0"):
        monkeypatch.setenv("MPCQP_LDS_CHAIN", on)
        h = OSQPBatch()
        h.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
        handles.append(h)
    monkeypatch.delenv("MPCQP_LDS_CHAIN")
    for step, kw in enumerate([dict(), dict(q=b["q"] * 1.01), dict(rho=0.3)]):
        for h in handles:
            if "rho" in kw:
                h.update_settings(**kw)
            elif kw:
                h.update(**kw)
        r1, r0 = handles[0].solve(), handles[1].solve()
        assert np.array_equal(r1.iter, r0.iter) and np.array_equal(r1.status_val, r0.status_val), step
        assert np.array_equal(r1.x, r0.x) and np.array_equal(r1.y, r0.y), step
        assert (r1.status_val == 1).all(), step


@pytest.mark.gpu
def test_long_horizon_reuse_after_a_rho_step_at_max_iter(monkeypatch):
    """a solve whose last iteration is a rho-adaptation step (max_iter a
    multiple of the rho interval) stores the new rho while the workspace factor is still the
    old rho's; the next solve must refactor (OSQP 0.6 refactors inside adapt_rho), not start
    from that stale factor.  cfg-5 handles that reuse the factor and ones that never do
    (MPCQP_FACTOR_REUSE=0) run max_iter = 100 / 200 / 300 cold, then two warm re-solves, and
    agree bit for bit; the rho step at the last iteration is confirmed to have fired on some
    instance (its rho-update count exceeds that of a max_iter - 1 run)."""
    b = mpc.make_batch(5, B=8, seed=21)
    P, A = b["P"], b["A"]
    fired = 0
    for mi in (100, 200, 300):
        s = dict(warm_start=True, polish=False, max_iter=mi)
        handles = []
        for reuse in ("1", "0"):
            monkeypatch.setenv("MPCQP_FACTOR_REUSE", reuse)
            h = OSQPBatch()
            h.setup(P, b["q"], A, b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
            handles.append(h)
        monkeypatch.setenv("MPCQP_FACTOR_REUSE", "0")
        short = OSQPBatch()
        short.setup(P, b["q"], A, b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **dict(s, max_iter=mi - 1))
        monkeypatch.delenv("MPCQP_FACTOR_REUSE")
        r1, r0, rs = handles[0].solve(), handles[1].solve(), short.solve()
        late = (r0.rho_updates > rs.rho_updates) & (r0.iter == mi)
        fired += int(late.sum())
        for step in range(3):
            assert np.array_equal(r1.iter, r0.iter) and np.array_equal(r1.status_val, r0.status_val), (mi, step)
            assert np.array_equal(r1.x, r0.x) and np.array_equal(r1.y, r0.y), (mi, step)
            if step < 2:
                r1, r0 = handles[0].solve(), handles[1].solve()
    assert fired > 0, "no instance adapted rho at its last iteration: the case is not exercised"


@pytest.mark.gpu
def test_long_horizon_middle_block_in_place(monkeypatch):
    """solve_big.hip::middle_apart: when the middle block's rows the top chain updates [0, amax)
    and the rows the bottom chain updates [toff_p, toff_p + bmax) are disjoint (cfg 5: rows 0-9
    and 20-29), the bottom chain writes (old - x) - y into rb in place (x, y: the last DPP
    level's two halves) and the middle step reads w_p alone; otherwise (MPCQP_MIDDLE_APART=0
    forces it) the bottom chain's x + y goes to corB and the middle step forms w_p - corB --
    the same update, rounded differently.  Both handles against the oracle doing the same
    calls (a cold solve, then a warm-started one after an update of q): statuses equal,
    iteration counts for >= 7/8 of the instances, and where they agree, the inputs within
    U_TOL; the two handles' iteration counts agree with each other as well."""
    b = mpc.make_batch(5, B=8, seed=23)
    s = dict(warm_start=True, polish=False)
    P, A = b["P"], b["A"]
    handles = []
    for apart in ("1", "0"):
        monkeypatch.setenv("MPCQP_MIDDLE_APART", apart)
        h = OSQPBatch()
        h.setup(P, b["q"], A, b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], **s)
        handles.append(h)
    monkeypatch.delenv("MPCQP_MIDDLE_APART")
    orc = []
    for k in range(b["Px"].shape[0]):
        o = pyoracle.OSQP()
        Pk, Ak = P.copy(), A.copy()
        Pk.data, Ak.data = b["Px"][k].copy(), b["Ax"][k].copy()
        o.setup(Pk, b["q"][k], Ak, b["l"][k], b["u"][k], **s)
        orc.append(o)
    for step in range(2):
        if step:
            for h in handles:
                h.update(q=b["q"] * 0.97)
            for k, o in enumerate(orc):
                o.update(q=b["q"][k] * 0.97)
        ro = [o.solve() for o in orc]
        it = np.array([r.info.iter for r in ro])
        st = np.array([r.info.status_val for r in ro])
        res = [h.solve() for h in handles]
        assert np.mean(res[0].iter == res[1].iter) >= 7 / 8, (step, res[0].iter, res[1].iter)
        for r in res:
            assert np.array_equal(r.status_val, st), (step, r.status_val, st)
            assert np.mean(r.iter == it) >= 7 / 8, (step, r.iter, it)
            same = r.iter == it
            du = np.array([np.abs(r.x[k, b["u_block"]] - ro[k].x[b["u_block"]]).max() for k in range(len(ro))])
            assert np.all(du[same] < U_TOL), (step, du[same].max())


@pytest.mark.gpu
def test_wide_setup_forms_and_fused_warm_start_agree(monkeypatch):
    """The wide batch setup (setup_wide.h): its 512-thread form (two instances per CU, batches of
    512 or more) and its 1024-thread form (MPCQP_SETUP_FULL=1), each as setup() + warm_start()
    and fused as setup_warm() (mpcqp_setup_warm_device: one kernel), give the same cfg-5 solve
    bit for bit -- with x0 and y0, and with x0 alone (y stays zero as warm_start leaves it)."""
    import torch
    from osqp_amd import DeviceBatch, _drop_common_zeros
    from osqp_amd.mpc_device import warm_shift
    B = 640
    b = mpc.make_batch(5, B=B, seed=41)
    P, Px = _drop_common_zeros(b["P"], b["Px"])
    A, Ax = _drop_common_zeros(b["A"], b["Ax"])
    s = {k: v for k, v in b["settings"].items() if k != "verbose"}
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    dPx, dAx, dq, dl, du = (t(a) for a in (Px, Ax, b["q"], b["l"], b["u"]))

    def outs():
        return (torch.empty((B, b["n"]), dtype=torch.float64, device=dev),
                torch.empty((B, b["m"]), dtype=torch.float64, device=dev),
                torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.int32, device=dev))

    h0 = DeviceBatch(P, A, B, device=0, **s)
    o = outs()
    h0.setup(dPx, dAx, dq, dl, du)
    h0.solve(*o)
    h0.synchronize()
    xs, ys = warm_shift(b["N"], 8, 2, o[0], o[1])
    torch.cuda.synchronize()
    for y0 in (ys, None):
        runs = []
        for full in ("0", "1"):
            monkeypatch.setenv("MPCQP_SETUP_FULL", full)
            for fused in (False, True):
                h = DeviceBatch(P, A, B, device=0, **s)
                assert h.setup_warm_fused() == 1
                o = outs()
                if fused:
                    h.setup_warm(dPx, dAx, dq, dl, du, xs, y0)
                else:
                    h.setup(dPx, dAx, dq, dl, du)
                    h.warm_start(xs, y0)
                h.solve(*o)
                h.synchronize()
                runs.append([v.cpu().numpy() for v in o])
        monkeypatch.delenv("MPCQP_SETUP_FULL")
        for r in runs[1:]:
            for a, c in zip(runs[0], r):
                assert np.array_equal(a.view(np.int64) if a.dtype == np.float64 else a,
                                      c.view(np.int64) if c.dtype == np.float64 else c)
        assert (runs[0][2] == 1).mean() > 0.99


@pytest.mark.gpu
def test_wide_setup_forms_agree_through_matrix_updates(monkeypatch):
    """A matrix update rescales through the wide setup's KEEP form (launch_update_mat): on a
    cfg-5 batch of 512 or more (its 512-thread form) and with MPCQP_SETUP_FULL=1 (the
    1024-thread form) the setup, a P update and an A update by index each solve to the same
    result bit for bit (test_matrix_updates_match_oracle holds the 1024-thread form to the
    oracle at B = 12)."""
    B = 520
    b = mpc.make_batch(5, B=B, seed=9)
    idx = np.concatenate([np.arange(0, b["A"].nnz, 3), [0]])
    An = b["Ax"][:, idx] * np.random.default_rng(3).uniform(0.99, 1.01, (B, idx.size))
    runs = []
    for full in ("0", "1"):
        monkeypatch.setenv("MPCQP_SETUP_FULL", full)
        dev = OSQPBatch()
        dev.setup(b["P"], b["q"], b["A"], b["l"], b["u"], Px=b["Px"], Ax=b["Ax"], warm_start=False)
        out = []
        for step in range(3):
            if step == 1:
                dev.update(Px=b["Px"] * 1.5)
            elif step == 2:
                dev.update(Ax=An, Ax_idx=idx)
            r = dev.solve()
            out.append((r.x.copy(), r.y.copy(), np.asarray(r.status_val).copy(), np.asarray(r.iter).copy()))
        runs.append(out)
    monkeypatch.delenv("MPCQP_SETUP_FULL")
    for a, c in zip(*runs):
        for u, v in zip(a, c):
            assert np.array_equal(u.view(np.int64) if u.dtype == np.float64 else u,
                                  v.view(np.int64) if v.dtype == np.float64 else v)
    assert (runs[0][0][2] == 1).mean() > 0.99
