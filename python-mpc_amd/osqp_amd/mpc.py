"""Host-side MPC -> QP assembly and batch generators.

The reference assembles each QP with scipy.sparse before calling
osqp.OSQP().setup() (the boundary this package replaces):

  * lateral slack + incremental MPC   vehicle_lateral_mpc_slack_increment.py:32-121 (+ loop :126-229)
  * vanilla LTI MPC                    Control/MPC/mpc_kinematics.py:148-200 (`mpc`)
  * incremental LTV MPC                Control/MPC/mpc_dynamics.py:281-389 (`mpc_increment`),
                                       Control/MPC/mpc_increment_kinematics_pred_matrix.py:150-240
  * dynamic-bicycle linearisation      Vehicle_Dynamics/vehicle_models.py:52-340 (`get_dynamics_model`)

The builders here produce the same matrices (tests/test_assembly.py checks
them entry-for-entry against tests/golden/, captured from the reference) with
the variable order the reference uses, x = (x_0..x_N, u_0..u_{N-1}[, s_0..s_N]).
Batch generators (`make_batch`) vectorise the same formulas over B instances
that share one sparsity pattern -- the synthetic workloads of BASELINE.json's
configs.  Everything here is host numpy: data preparation,
not the solver.
"""
from __future__ import annotations

import math

import numpy as np
import scipy.sparse as sparse

# ------------------------------------------------------------------ models --
LATERAL_AD = np.array([[0.960, -0.019, 0., 0.],
                       [0.00469, 0.961, 0., 0.],
                       [0., 0.0196, 1., 0.],
                       [0.163, 0., 0.166, 1.]])          # slack script :32-37 (beta, r, e_psi, e_y)
LATERAL_BD = np.array([[0.020575], [0.115], [0.001157], [0.00182]])  # :39-43


def augment(Ad, Bd):
    """Incremental-input augmentation  x~ = [x; u_prev]:  A~ = [[Ad, Bd], [0, I]],  B~ = [Bd; I]
    (slack script :48-52, mpc_dynamics.py:333-361)."""
    nx, nu = Bd.shape
    At = np.block([[Ad, Bd], [np.zeros((nu, nx)), np.eye(nu)]])
    Bt = np.vstack([Bd, np.eye(nu)])
    return At, Bt


def _csc(M):
    M = sparse.csc_matrix(M)
    M.eliminate_zeros()
    M.sort_indices()
    return M


def _dyn_eq(Ad_list, Bd_list, N):
    """[-I stacked on the diagonal | A_k on the sub-diagonal | B_k shifted one block down]."""
    nx = Ad_list[0].shape[0]
    nu = Bd_list[0].shape[1]
    Ax = sparse.kron(sparse.eye(N + 1), -sparse.eye(nx), format="lil")
    Bu = sparse.lil_matrix(((N + 1) * nx, N * nu))
    for k in range(N):
        Ax[(k + 1) * nx:(k + 2) * nx, k * nx:(k + 1) * nx] = Ad_list[k]
        Bu[(k + 1) * nx:(k + 2) * nx, k * nu:(k + 1) * nu] = Bd_list[k]
    return sparse.hstack([Ax, Bu]).tocsc()


# ------------------------------------------------------- vanilla (cfg 2) --
def vanilla_qp(Ad, Bd, gd, x0, Xr, Q, QN, R, N, xmin, xmax, umin, umax):
    """Control/MPC/mpc_kinematics.py:148-191 (`mpc`): returns P, q, A, l, u."""
    Ad = np.asarray(Ad, float); Bd = np.asarray(Bd, float)
    nx, nu = Bd.shape
    Q = np.asarray(sparse.csr_matrix(Q).todense()); QN = np.asarray(sparse.csr_matrix(QN).todense())
    R = np.asarray(sparse.csr_matrix(R).todense())
    P = sparse.block_diag([sparse.kron(sparse.eye(N), Q), QN, sparse.kron(sparse.eye(N), R)])
    q = np.concatenate([-(Q @ Xr[:, k]) for k in range(N)] + [-(QN @ Xr[:, N]), np.zeros(N * nu)])
    Aeq = _dyn_eq([Ad] * N, [Bd] * N, N)
    gd = np.asarray(gd, float).ravel()
    leq = np.concatenate([-np.asarray(x0, float)] + [-gd] * N)
    Aineq = sparse.eye((N + 1) * nx + N * nu)
    lineq = np.concatenate([np.tile(xmin, N + 1), np.tile(umin, N)])
    uineq = np.concatenate([np.tile(xmax, N + 1), np.tile(umax, N)])
    A = sparse.vstack([Aeq, Aineq])
    return _csc(P), q, _csc(A), np.concatenate([leq, lineq]), np.concatenate([leq, uineq])


# ---------------------------------------------------------- slack (cfg 1/3/4) --
SLACK_Q = np.diag([5., 5., 10., 10.])                        # :66
SLACK_R = 10.0                                               # :71
SLACK_W = np.array([10., 10., 10., 10., 0.])                 # :73 (0: the u_prev slot)
SLACK_WS = np.array([1., 1., 1., 1., 0.])                    # :104 slack coefficients
DEG = np.pi / 180.0


def slack_bounds(regime=0):
    """Bound schedule of the slack script :158-172 (regime 0: i<=400 / i>900, 1: 400<i<=900)."""
    dumin = np.array([-0.5 * DEG]); dumax = np.array([0.5 * DEG])
    xmin = np.array([-np.pi, -0.5 * np.pi, -15 * DEG, -10., -30 * DEG])
    xmax = np.array([np.pi, 0.5 * np.pi, 15 * DEG, 10., 30 * DEG])
    if regime == 1:
        xmin = xmin.copy(); xmin[3] = 2.0
    return xmin, xmax, dumin, dumax


def slack_qp(N, x0, xr=None, regime=0):
    """vehicle_lateral_mpc_slack_increment.py:48-115: soft-constrained incremental lateral MPC.
    Variables (x~_0..x~_N, du_0..du_{N-1}, s_0..s_N)."""
    At, Bt = augment(LATERAL_AD, LATERAL_BD)
    nx, nu = Bt.shape                                   # 5, 1
    nxs = nx - nu
    xr = np.zeros(nxs) if xr is None else np.asarray(xr, float)
    C = np.hstack([np.eye(nxs), np.zeros((nxs, nu))])
    Qt = C.T @ SLACK_Q @ C
    P = sparse.block_diag([sparse.kron(sparse.eye(N + 1), Qt), sparse.kron(sparse.eye(N), SLACK_R * np.eye(nu)),
                           sparse.kron(sparse.eye(N + 1), np.diag(SLACK_W))])
    qx = -(SLACK_Q @ C).T @ xr
    q = np.concatenate([np.tile(qx, N + 1), np.zeros(N * nu), np.zeros((N + 1) * nx)])
    Aeq = sparse.hstack([_dyn_eq([At] * N, [Bt] * N, N), sparse.csc_matrix(((N + 1) * nx, (N + 1) * nx))])
    Sineq = sparse.vstack([sparse.kron(sparse.eye(N + 1), np.diag(SLACK_WS)), sparse.csc_matrix((N * nu, (N + 1) * nx))])
    Aineq = sparse.hstack([sparse.eye((N + 1) * nx + N * nu), Sineq])
    xmin, xmax, dumin, dumax = slack_bounds(regime)
    leq = np.concatenate([-np.asarray(x0, float), np.zeros(N * nx)])
    lineq = np.concatenate([np.tile(xmin, N + 1), np.tile(dumin, N)])
    uineq = np.concatenate([np.tile(xmax, N + 1), np.tile(dumax, N)])
    A = sparse.vstack([Aeq, Aineq])
    return _csc(P), q, _csc(A), np.concatenate([leq, lineq]), np.concatenate([leq, uineq])


# ------------------------------------------------------- incremental LTV (cfg 5) --
def incremental_qp(Ad_list, Bd_list, gd_list, xt0, Xr, Q, QN, R, N, xmin_t, xmax_t, dumin, dumax):
    """Control/MPC/mpc_dynamics.py:281-389 (`mpc_increment`): augmented LTV MPC in increments."""
    nx = Ad_list[0].shape[0]
    nu = Bd_list[0].shape[1]
    Q = np.asarray(sparse.csr_matrix(Q).todense()); QN = np.asarray(sparse.csr_matrix(QN).todense())
    R = np.asarray(sparse.csr_matrix(R).todense())
    C = np.hstack([np.eye(nx), np.zeros((nx, nu))])
    P = sparse.block_diag([sparse.kron(sparse.eye(N), C.T @ Q @ C), C.T @ QN @ C, sparse.kron(sparse.eye(N), R)])
    q = np.concatenate([-(Q @ C).T @ Xr[:, k] for k in range(N)] + [-(QN @ C).T @ Xr[:, N], np.zeros(N * nu)])
    aug = [augment(np.asarray(Ad_list[k], float), np.asarray(Bd_list[k], float)) for k in range(N)]
    Aeq = _dyn_eq([a[0] for a in aug], [a[1] for a in aug], N)
    gt = [np.concatenate([np.asarray(gd_list[k], float).ravel(), np.zeros(nu)]) for k in range(N)]
    leq = np.concatenate([-np.asarray(xt0, float)] + [-g for g in gt])
    Aineq = sparse.eye((N + 1) * (nx + nu) + N * nu)
    lineq = np.concatenate([np.tile(xmin_t, N + 1), np.tile(dumin, N)])
    uineq = np.concatenate([np.tile(xmax_t, N + 1), np.tile(dumax, N)])
    A = sparse.vstack([Aeq, Aineq])
    return _csc(P), q, _csc(A), np.concatenate([leq, lineq]), np.concatenate([leq, uineq])


# ------------------------------------------------ dynamic bicycle linearisation --
class VehicleParams:
    """Vehicle_Dynamics.__init__ (vehicle_models.py:27-50) defaults, dt as in mpc_dynamics.main (0.05)."""

    def __init__(self, m=1300, l_f=1.25, l_r=1.40, width=1.78, length=4.25, turning_circle=10.4,
                 C_d=0.34, A_f=2.0, C_roll=0.015, dt=0.05):
        self.m, self.l_f, self.l_r, self.dt = m, l_f, l_r, dt
        self.wheelbase = l_f + l_r
        self.Iz = 1 / 12 * m * (width ** 2 + length ** 2)
        self.C_d, self.A_f, self.C_roll, self.roh = C_d, A_f, C_roll, 1.23

    def pacejka(self):
        """Lateral Pacejka coefficients (vehicle_models.py:114-132): (B, C, D) front and rear."""
        a = [-22.1, 1011, 1078, 1.82, 0.208, 0.000, -0.354, 0.707]
        out = []
        for share in (self.l_r, self.l_f):
            Fz = 9.81 * (self.m * share / self.wheelbase) * 0.001
            C = 1.30
            D = a[0] * Fz ** 2 + a[1] * Fz
            BCD = a[2] * math.sin(a[3] * math.atan(a[4] * Fz))
            out.append((BCD / (C * D) * 180 / np.pi, C, D))
        return out


def linearise_dynamics(veh: VehicleParams, x, u):
    """Batched forward-Euler linearisation of the dynamic bicycle model
    (vehicle_models.py:52-340): x (B,6) = [X, Y, yaw, vx, vy, r], u (B,2) = [steer, accel]
    -> Ad (B,6,6), Bd (B,6,2), gd (B,6).  Applies the low-speed guard of :143-159
    to copies (the reference mutates the caller's arrays there)."""
    x = np.array(x, float, copy=True); u = np.array(u, float, copy=True)
    vx = x[:, 3]
    g1 = (vx >= 0) & (vx < 0.5)
    g2 = (vx > -0.5) & (vx < 0)
    g = g1 | g2
    x[g, 4] = 0.0; x[g, 5] = 0.0; u[g, 0] = 0.0
    x[g1 & (vx < 0.3), 3] = 0.3
    x[g2 & (vx > -0.3), 3] = -0.3
    (Bf, Cf, Df), (Br, Cr, Dr) = veh.pacejka()
    m, Iz, lf, lr = veh.m, veh.Iz, veh.l_f, veh.l_r
    yaw, vx, vy, r = x[:, 2], x[:, 3], x[:, 4], x[:, 5]
    st, acc = u[:, 0], u[:, 1]
    af = -np.arctan2(lf * r + vy, vx) + st
    ar = -np.arctan2(-lr * r + vy, vx)
    Fyf = Df * np.sin(Cf * np.arctan(Bf * af))
    Fyr = Dr * np.sin(Cr * np.arctan(Br * ar))
    R_roll = veh.C_roll * m * 9.81 * np.sign(vx)
    F_aero = 0.5 * veh.roh * veh.C_d * veh.A_f * vx ** 2 * np.sign(vx)
    Fx = m * acc - F_aero - R_roll
    cy, sy, cs, ss = np.cos(yaw), np.sin(yaw), np.cos(st), np.sin(st)
    f = np.stack([vx * cy - vy * sy, vy * cy + vx * sy, r,
                  1. / m * (Fx * cs - Fyf * ss + m * vy * r),
                  1. / m * (Fx * ss + Fyr + Fyf * cs - m * vx * r),
                  1. / Iz * (Fx * lf * ss + Fyf * lf * cs - Fyr * lr)], axis=1)
    dFx_dvx = -veh.roh * veh.C_d * veh.A_f * vx
    dFx_da = m
    kf = (Bf * Cf * Df * np.cos(Cf * np.arctan(Bf * af))) / (1 + Bf ** 2 * af ** 2)
    kr = (Br * Cr * Dr * np.cos(Cr * np.arctan(Br * ar))) / (1 + Br ** 2 * ar ** 2)
    nf = (lf * r + vy) ** 2 + vx ** 2
    nr = (-lr * r + vy) ** 2 + vx ** 2
    dFyf_dvx = kf * (lf * r + vy) / nf
    dFyf_dvy = kf * (-vx / nf)
    dFyf_dr = kf * (-lf * vx) / nf
    dFyf_dst = kf
    dFyr_dvx = kr * (-lr * r + vy) / nr
    dFyr_dvy = kr * (-vx) / nr
    dFyr_dr = kr * (lr * vx) / nr
    B = x.shape[0]
    Ac = np.zeros((B, 6, 6))
    Ac[:, 0, 2] = -vx * sy - vy * cy; Ac[:, 0, 3] = cy; Ac[:, 0, 4] = -sy
    Ac[:, 1, 2] = -vy * sy + vx * cy; Ac[:, 1, 3] = sy; Ac[:, 1, 4] = cy
    Ac[:, 2, 5] = 1.
    Ac[:, 3, 3] = 1 / m * (dFx_dvx * cs - dFyf_dvx * ss)
    Ac[:, 3, 4] = 1 / m * (-dFyf_dvy * ss + m * r)
    Ac[:, 3, 5] = 1 / m * (-dFyf_dr * ss + m * vy)
    Ac[:, 4, 3] = 1 / m * (dFx_dvx * ss + dFyr_dvx + dFyf_dvx * cs - m * r)
    Ac[:, 4, 4] = 1 / m * (dFyr_dvy + dFyf_dvy * cs)
    Ac[:, 4, 5] = 1 / m * (dFyr_dr + dFyf_dr * cs - m * vx)
    Ac[:, 5, 3] = 1 / Iz * (dFx_dvx * lf * ss + dFyf_dvx * lf * cs - dFyr_dvx * lr)
    Ac[:, 5, 4] = 1 / Iz * (dFyf_dvy * lf * cs - dFyr_dvy * lr)
    Ac[:, 5, 5] = 1 / Iz * (dFyf_dr * lf * cs - dFyr_dr * lr)
    Bc = np.zeros((B, 6, 2))
    Bc[:, 3, 0] = 1 / m * (-Fx * ss - dFyf_dst * ss - Fyf * cs)
    Bc[:, 3, 1] = 1 / m * (dFx_da * cs)
    Bc[:, 4, 0] = 1 / m * (Fx * cs + dFyf_dst * cs - Fyf * ss)
    Bc[:, 4, 1] = 1 / m * (dFx_da * ss)
    Bc[:, 5, 0] = 1 / Iz * (Fx * lf * cs + dFyf_dst * lf * cs - Fyf * lf * ss)
    Bc[:, 5, 1] = 1 / Iz * (dFx_da * lf * ss)
    gc = f - np.einsum("bij,bj->bi", Ac, x) - np.einsum("bij,bj->bi", Bc, u)
    Ad = np.eye(6)[None] + Ac * veh.dt
    return Ad, Bc * veh.dt, gc * veh.dt


# ------------------------------------------------------------ batch generators --
CONFIGS = {
    1: dict(name="slack-single-N20", layout="slack", N=20, B=1),
    2: dict(name="vanilla-lateral-N20", layout="vanilla", N=20, B=1024),
    3: dict(name="slack-lateral-N20", layout="slack", N=20, B=65536),
    4: dict(name="slack-lateral-N20-8gpu", layout="slack", N=20, B=262144),
    5: dict(name="incremental-dynamic-N50", layout="dynamic", N=50, B=8192),
}

VANILLA_Q = np.diag([5., 5., 10., 10.])
VANILLA_R = np.array([[10.]])
VANILLA_XMIN = np.array([-np.pi, -0.5 * np.pi, -15 * DEG, -10.])
VANILLA_UMAX = np.array([30 * DEG])

DYN_Q = np.diag([100.0, 100.0, 100.0, 50.0, 50.0, 50.0])        # mpc_dynamics.py:456-458
DYN_QN = np.diag([1000.0, 1000.0, 1000.0, 500.0, 500.0, 500.0])
DYN_R = np.diag([50., 50.])
DYN_DUMIN = np.array([-np.deg2rad(2.0), -0.5])                   # :461-464
DYN_XMIN_T = np.array([-np.inf, -np.inf, -2 * np.pi, -100., -30., -0.5 * np.pi, -np.deg2rad(15), -3.])
DYN_XMAX_T = np.array([np.inf, np.inf, 2 * np.pi, 100., 30., 0.5 * np.pi, np.deg2rad(15), 1.])


def _lateral_x0(rng, B):
    return np.stack([rng.uniform(-.05, .05, B), rng.uniform(-.1, .1, B), rng.uniform(-10, 10, B) * DEG,
                     rng.uniform(-3, 3, B)], axis=1)


def make_batch(cfg: int, B: int | None = None, seed: int | None = None, N: int | None = None):
    """Synthetic batch for BASELINE.json config `cfg`.

    Returns dict(P, A: scipy CSC templates (shared pattern), Px (B,nnzP), Ax (B,nnzA),
    q (B,n), l (B,m), u (B,m), n, m, N, u_slice (slice of the first control in x),
    name, settings (the reference call site's osqp keywords))."""
    spec = CONFIGS[cfg]
    B = spec["B"] if B is None else B
    N = spec["N"] if N is None else N
    rng = np.random.default_rng(cfg if seed is None else seed)
    layout = spec["layout"]
    if layout == "vanilla":
        x0 = _lateral_x0(rng, B)
        P, q0, A, l0, u0 = vanilla_qp(LATERAL_AD, LATERAL_BD, np.zeros(4), np.zeros(4), np.zeros((4, N + 1)),
                                      VANILLA_Q, VANILLA_Q, VANILLA_R, N, VANILLA_XMIN, -VANILLA_XMIN,
                                      -VANILLA_UMAX, VANILLA_UMAX)
        nx, nu = 4, 1
        l = np.tile(l0, (B, 1)); u = np.tile(u0, (B, 1))
        l[:, :nx] = -x0; u[:, :nx] = -x0
        q = np.tile(q0, (B, 1))
        Px = np.tile(P.data, (B, 1)); Ax = np.tile(A.data, (B, 1))
        ucol = (N + 1) * nx
        settings = dict(verbose=False, warm_start=True)           # mpc_kinematics.py:195
        theta = np.concatenate([x0, np.zeros((B, 4 * (N + 1)))], axis=1)  # (x0, Xr): mpc_device.LateralAssembler
        regime = np.zeros(B, np.int32)
    elif layout == "slack":
        nx, nu = 5, 1
        x0 = np.concatenate([_lateral_x0(rng, B), rng.uniform(-5, 5, (B, 1)) * DEG], axis=1)
        P, q0, A, l0, u0 = slack_qp(N, np.zeros(nx))
        _, _, _, l1, _ = slack_qp(N, np.zeros(nx), regime=1)
        reg = rng.uniform(size=B) < 0.3                            # e_y >= 2 regime (:163-167)
        l = np.where(reg[:, None], l1[None], l0[None]).copy(); u = np.tile(u0, (B, 1))
        l[:, :nx] = -x0; u[:, :nx] = -x0
        q = np.tile(q0, (B, 1))
        Px = np.tile(P.data, (B, 1)); Ax = np.tile(A.data, (B, 1))
        ucol = (N + 1) * nx
        settings = dict(warm_start=True)                           # slack script :121
        theta = np.concatenate([x0, np.zeros((B, 4))], axis=1)     # (x~0, xr): mpc_device.LateralAssembler
        regime = reg.astype(np.int32)
    elif layout == "dynamic":
        veh = VehicleParams(dt=0.05)
        nx, nu = 6, 2
        xs = np.zeros((B, 6))
        xs[:, 2] = rng.uniform(-np.pi / 8, np.pi / 8, B)
        xs[:, 3] = rng.uniform(5, 25, B)
        xs[:, 4] = rng.uniform(-.5, .5, B)
        xs[:, 5] = rng.uniform(-.2, .2, B)
        us = np.stack([np.deg2rad(rng.uniform(-5, 5, B)), rng.uniform(-1, 1, B)], axis=1)
        yoff = rng.uniform(-4, 4, B)
        Ads, Bds, gds = [], [], []
        xk = xs.copy()
        for k in range(N):                                         # zero-increment rollout (:506-514)
            Ad, Bd, gd = linearise_dynamics(veh, xk, us)
            Ads.append(Ad); Bds.append(Bd); gds.append(gd)
            xk = np.einsum("bij,bj->bi", Ad, xk) + np.einsum("bij,bj->bi", Bd, us) + gd
        Ads = np.stack(Ads, 1); Bds = np.stack(Bds, 1); gds = np.stack(gds, 1)
        Xr = np.zeros((B, 6, N + 1))
        Xr[:, 0] = np.arange(N + 1)[None] * 10.0 * 0.05
        Xr[:, 1] = yoff[:, None]
        Xr[:, 3] = 10.0
        xt0 = np.concatenate([xs, us], axis=1)
        # shared pattern: every entry of Ad / Bd that is nonzero for some instance or stage
        maskA = np.abs(Ads).max(axis=(0, 1)) > 0
        maskB = np.abs(Bds).max(axis=(0, 1)) > 0
        P, _, A, _, _ = incremental_qp([np.where(maskA, 7.0, 0.0)] * N, [np.where(maskB, 7.0, 0.0)] * N,
                                       [np.zeros(6)] * N, np.zeros(8), np.zeros((6, N + 1)), DYN_Q, DYN_QN, DYN_R,
                                       N, DYN_XMIN_T, DYN_XMAX_T, DYN_DUMIN, -DYN_DUMIN)
        pa, pb, pb2 = _stage_positions(A, N, nx, nu, maskA, maskB)
        Ax = np.tile(A.data, (B, 1))
        ii, jj = np.nonzero(maskA)
        Ax[:, pa] = Ads[:, :, ii, jj].reshape(B, -1)
        ii2, jj2 = np.nonzero(maskB)
        Ax[:, pb] = Bds[:, :, ii2, jj2].reshape(B, -1)
        Ax[:, pb2] = Bds[:, :, ii2, jj2].reshape(B, -1)
        Px = np.tile(P.data, (B, 1))
        C = np.hstack([np.eye(nx), np.zeros((nx, nu))])
        qx = -np.einsum("ij,bjk->bki", (DYN_Q @ C).T, Xr[:, :, :N])
        qN = -np.einsum("ij,bj->bi", (DYN_QN @ C).T, Xr[:, :, N])
        q = np.concatenate([qx.reshape(B, -1), qN, np.zeros((B, N * nu))], axis=1)
        n_x = (N + 1) * (nx + nu)
        gt = np.concatenate([gds, np.zeros((B, N, nu))], axis=2).reshape(B, -1)
        leq = np.concatenate([-xt0, -gt], axis=1)
        lineq = np.concatenate([np.tile(DYN_XMIN_T, N + 1), np.tile(DYN_DUMIN, N)])
        uineq = np.concatenate([np.tile(DYN_XMAX_T, N + 1), np.tile(-DYN_DUMIN, N)])
        l = np.concatenate([leq, np.tile(lineq, (B, 1))], axis=1)
        u = np.concatenate([leq, np.tile(uineq, (B, 1))], axis=1)
        ucol = n_x
        settings = dict(verbose=True, polish=False, warm_start=False)   # mpc_dynamics.py:393
        theta = regime = None
    else:
        raise ValueError(layout)
    n, m = P.shape[0], A.shape[0]
    return dict(P=P, A=A, Px=np.ascontiguousarray(Px), Ax=np.ascontiguousarray(Ax), q=np.ascontiguousarray(q),
                l=np.ascontiguousarray(l), u=np.ascontiguousarray(u), n=n, m=m, N=N, B=B, nu=nu,
                u_slice=slice(ucol, ucol + nu), u_block=slice(ucol, ucol + N * nu), name=spec["name"],
                settings=settings, cfg=cfg, theta=theta, regime=regime)


def _stage_positions(A, N, nx, nu, maskA, maskB):
    """Indices into A.data of the Ad entries of A~_k, of the Bd entries of A~_k (u_prev
    columns) and of the Bd entries of B~_k (du_k columns), ordered (stage, mask nonzero)."""
    A = A.tocsc()
    nxa = nx + nu
    ncol_x = (N + 1) * nxa

    def pos(r, c):
        lo, hi = A.indptr[c], A.indptr[c + 1]
        k = lo + np.searchsorted(A.indices[lo:hi], r)
        assert k < hi and A.indices[k] == r, (r, c)
        return k

    ii, jj = np.nonzero(maskA)
    ii2, jj2 = np.nonzero(maskB)
    pa, pb = [], []
    for k in range(N):
        r0 = (k + 1) * nxa
        for i, j in zip(ii, jj):
            pa.append(pos(r0 + i, k * nxa + j))
        for i, j in zip(ii2, jj2):
            # Bd appears twice per stage: in A~ (column of u_prev) and in B~ (column of du_k).
            pb.append(pos(r0 + i, k * nxa + nx + j))
    pb2 = []
    for k in range(N):
        r0 = (k + 1) * nxa
        for i, j in zip(ii2, jj2):
            pb2.append(pos(r0 + i, ncol_x + k * nu + j))
    return np.array(pa), np.array(pb), np.array(pb2)
