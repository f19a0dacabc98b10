"""Device-resident MPC data path around the solver.

The reference's incremental dynamic-bicycle MPC (Control/MPC/mpc_dynamics.py:main)
does, per control step and in Python:

  Xr = reference_search(path_x, path_y, pred_x~, dt, N)            :44-90   (F3)
  Ad_k, Bd_k, gd_k = vehicle.get_dynamics_model(pred_x~[:, k])      vehicle_models.py:52-340 (F2)
  pred_x~, pred_du = mpc_increment(Ad, Bd, gd, x~, Xr, ...)         :281-432 (F1 + the solve)
  plant step + horizon shift                                        :578-617 (F3)

This module runs the same steps for B vehicles at once on the MI355X through the
C ABI of include/mpcqp.h (mpcqp_linearise_device, mpcqp_incr_*,
mpcqp_reference_search_device) and the batched solver (DeviceBatch).  Arrays are
torch tensors on the device; nothing is copied to the host inside a step.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import scipy.sparse as sparse

from . import DeviceBatch, _check, lib

_P = C.POINTER
vp = C.c_void_p


class Vehicle(C.Structure):
    """Vehicle_Dynamics.__init__ arguments (vehicle_models.py:27-50); dt as in mpc_dynamics.main (0.05)."""
    _fields_ = [(k, C.c_double) for k in ("m", "l_f", "l_r", "width", "length", "C_d", "A_f", "C_roll", "dt")]

    def __init__(self, m=1300, l_f=1.25, l_r=1.40, width=1.78, length=4.25, C_d=0.34, A_f=2.0, C_roll=0.015,
                 dt=0.05):
        super().__init__(m, l_f, l_r, width, length, C_d, A_f, C_roll, dt)


# structural nonzeros of get_dynamics_model's Ad = I + dt Ac and Bd = dt Bc (vehicle_models.py:273-292)
DYN_MASK_A = np.eye(6, dtype=np.uint8)
for _i, _j in [(0, 2), (0, 3), (0, 4), (1, 2), (1, 3), (1, 4), (2, 5), (3, 3), (3, 4), (3, 5), (4, 3), (4, 4),
               (4, 5), (5, 3), (5, 4), (5, 5)]:
    DYN_MASK_A[_i, _j] = 1
DYN_MASK_B = np.zeros((6, 2), np.uint8)
DYN_MASK_B[3:, :] = 1


def _bind():
    L = lib()
    if getattr(L, "_mpc_bound", False):
        return L
    i64, i32, d = C.c_int64, C.c_int32, C.c_double
    L.mpcqp_linearise_device.argtypes = [_P(Vehicle), i64, i32, vp, i64, i64, vp, i64, i64, vp, vp, vp, i32, vp]
    L.mpcqp_incr_layout_create.argtypes = [i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, _P(vp)]
    L.mpcqp_incr_layout_dims.argtypes = [vp, _P(i32), _P(i32), _P(i32), _P(i32)]
    L.mpcqp_incr_layout_pattern.argtypes = [vp] * 9
    L.mpcqp_incr_assemble_device.argtypes = [vp, i64] + [vp] * 10
    L.mpcqp_incr_layout_free.argtypes = [vp]
    L.mpcqp_incr_layout_free.restype = None
    L.mpcqp_reference_search_device.argtypes = [i64, i32, i32, i32, vp, vp, vp, d, vp, i32, vp]
    L.mpcqp_incr_shift_device.argtypes = [vp, _P(Vehicle), i64, vp, vp, vp, vp, vp, vp, vp, vp]
    L.mpcqp_incr_warm_shift_device.argtypes = [i64, i32, i32, i32, vp, vp, vp, vp, i32, vp]
    L.mpcqp_affine_create.argtypes = [i32, vp, i32, i32, vp, vp, vp, i32, _P(vp)]
    L.mpcqp_affine_apply_device.argtypes = [vp, i64, vp, i32, vp, vp, vp, vp, vp]
    L.mpcqp_affine_free.argtypes = [vp]
    L.mpcqp_affine_free.restype = None
    L._mpc_bound = True
    return L


def _p(t):
    return C.c_void_p(t.data_ptr())


def _np_ptr(a):
    return C.c_void_p(a.ctypes.data)


def _stream(torch, device):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def linearise(veh: Vehicle, x, u, device=0):
    """Batched Vehicle_Dynamics.get_dynamics_model (F2).

    x: (B, N, 6) or (B, 6) float64 device tensor, u: (B, N, 2) or (B, 2) (any strides
    with a contiguous last dimension) -> Ad (B, N, 6, 6), Bd (B, N, 6, 2), gd (B, N, 6)
    (N axis dropped for 2-D inputs).  Inputs are not modified (the reference's
    low-speed guard writes into the caller's view; here it acts on copies)."""
    import torch
    L = _bind()
    squeeze = x.dim() == 2
    if squeeze:
        x, u = x[:, None, :], u[:, None, :]
    B, N = x.shape[0], x.shape[1]
    if x.shape[2] != 6 or u.shape[2] != 2 or u.shape[:2] != x.shape[:2]:
        raise ValueError("x must be (B, N, 6) and u (B, N, 2)")
    if x.stride(2) != 1 or u.stride(2) != 1:
        raise ValueError("the state / input axis must be contiguous")
    kw = dict(dtype=torch.float64, device=x.device)
    Ad = torch.empty((B, N, 6, 6), **kw); Bd = torch.empty((B, N, 6, 2), **kw); gd = torch.empty((B, N, 6), **kw)
    _check(L.mpcqp_linearise_device(C.byref(veh), B, N, _p(x), x.stride(0), x.stride(1), _p(u), u.stride(0),
                                    u.stride(1), _p(Ad), _p(Bd), _p(gd), x.device.index or 0,
                                    _stream(torch, x.device)), "linearise")
    if squeeze:
        return Ad[:, 0], Bd[:, 0], gd[:, 0]
    return Ad, Bd, gd


class IncrementalLayout:
    """The QP of mpc_increment (mpc_dynamics.py:281-389) for a batch sharing N, weights,
    bounds and the structural nonzeros of Ad / Bd (F1).  ``pattern()`` gives the CSC
    templates (P with its values, A), ``assemble()`` the per-instance values on the device."""

    def __init__(self, N, Q, QN, R, xmin_t, xmax_t, dumin, dumax, maskA=DYN_MASK_A, maskB=DYN_MASK_B, device=0):
        L = _bind()
        Q = np.ascontiguousarray(np.asarray(sparse.csr_matrix(Q).todense(), np.float64))
        QN = np.ascontiguousarray(np.asarray(sparse.csr_matrix(QN).todense(), np.float64))
        R = np.ascontiguousarray(np.asarray(sparse.csr_matrix(R).todense(), np.float64))
        self.N, self.nx, self.nu = int(N), Q.shape[0], R.shape[0]
        self.nxa = self.nx + self.nu
        arrs = [np.ascontiguousarray(np.asarray(a, np.float64).ravel()) for a in (xmin_t, xmax_t, dumin, dumax)]
        mA = np.ascontiguousarray(np.asarray(maskA, np.uint8))
        mB = np.ascontiguousarray(np.asarray(maskB, np.uint8))
        h = C.c_void_p()
        _check(L.mpcqp_incr_layout_create(self.N, self.nx, self.nu, _np_ptr(Q), _np_ptr(QN), _np_ptr(R),
                                          *(_np_ptr(a) for a in arrs), _np_ptr(mA), _np_ptr(mB), int(device),
                                          C.byref(h)), "incr_layout_create")
        self._h = h.value
        self._free = L.mpcqp_incr_layout_free  # held: module globals may be gone at interpreter exit
        self._keep = (Q, QN, R, arrs, mA, mB)
        n, m, nP, nA = (C.c_int32() for _ in range(4))
        _check(L.mpcqp_incr_layout_dims(self._h, C.byref(n), C.byref(m), C.byref(nP), C.byref(nA)), "dims")
        self.n, self.m, self.nnzP, self.nnzA = n.value, m.value, nP.value, nA.value
        self.device = int(device)

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            self._free(h)

    def pattern(self):
        """(P, A, l_template, u_template): scipy CSC templates (P upper triangle with its
        constant values; A with the constant entries and zeros at the stage entries) and
        the inequality-row bounds (clipped to +-1e30; equality rows 0)."""
        n, m = self.n, self.m
        Pp = np.zeros(n + 1, np.int32); Pi = np.zeros(self.nnzP, np.int32); Px = np.zeros(self.nnzP)
        Ap = np.zeros(n + 1, np.int32); Ai = np.zeros(self.nnzA, np.int32); At = np.zeros(self.nnzA)
        lt = np.zeros(m); ut = np.zeros(m)
        _check(lib().mpcqp_incr_layout_pattern(self._h, *(_np_ptr(a) for a in (Pp, Pi, Px, Ap, Ai, At, lt, ut))),
               "pattern")
        P = sparse.csc_matrix((Px, Pi, Pp), shape=(n, n))
        A = sparse.csc_matrix((At, Ai, Ap), shape=(m, n))
        return P, A, lt, ut

    def assemble(self, Ad, Bd, gd, xt0, Xr, out=None):
        """Ad (B,N,nx,nx), Bd (B,N,nx,nu), gd (B,N,nx), xt0 (B,nx+nu), Xr (B,nx,N+1), all
        contiguous float64 device tensors -> (Ax, q, l, u) in the layout's pattern order."""
        import torch
        B = Ad.shape[0]
        if out is None:
            kw = dict(dtype=torch.float64, device=Ad.device)
            out = (torch.empty((B, self.nnzA), **kw), torch.empty((B, self.n), **kw),
                   torch.empty((B, self.m), **kw), torch.empty((B, self.m), **kw))
        for t in (Ad, Bd, gd, xt0, Xr):
            if not t.is_contiguous() or t.dtype != torch.float64:
                raise ValueError("assemble inputs must be contiguous float64 tensors")
        Ax, q, l, u = out
        _check(lib().mpcqp_incr_assemble_device(self._h, B, _p(Ad), _p(Bd), _p(gd), _p(xt0), _p(Xr), _p(Ax), _p(q),
                                                _p(l), _p(u), _stream(torch, Ad.device)), "incr_assemble")
        return out


class AffineMap:
    """v = base[regime] + sum_t coef[:, t] * theta[idx[:, t]] over the concatenated (q | l | u)
    of an LTI layout -- the host description of mpcqp_affine (include/mpcqp.h), built by
    probing an assembler that is affine in theta: base[r] = build(0, r), and the terms of
    entry i from build(e_k, 0) for each parameter k.  `evaluate` applies it on the host
    (the CPU tests' check of the map against the builder); `LateralAssembler` uploads it."""

    def __init__(self, build, nparam, nregimes):
        outs0 = [np.concatenate(build(np.zeros(nparam), r)) for r in range(nregimes)]
        self.seglen = [len(v) for v in build(np.zeros(nparam), 0)]
        self.base = np.ascontiguousarray(np.stack(outs0))
        cols = []
        for k in range(nparam):
            e = np.zeros(nparam)
            e[k] = 1.0
            cols.append(np.concatenate(build(e, 0)) - outs0[0])
        Cm = np.stack(cols, axis=1) if cols else np.zeros((self.base.shape[1], 0))
        L = Cm.shape[0]
        nz = [np.flatnonzero(Cm[i]) for i in range(L)]
        self.T = max([len(z) for z in nz] + [0])
        self.idx = np.full((L, max(self.T, 1)), -1, np.int32)
        self.coef = np.zeros((L, max(self.T, 1)))
        for i, z in enumerate(nz):
            self.idx[i, :len(z)] = z
            self.coef[i, :len(z)] = Cm[i, z]
        # an entry that varies with theta has the same base in every regime (bounds change only
        # on constant rows), so one affine form per entry covers every regime
        var = np.array([len(z) > 0 for z in nz])
        if var.any() and not np.all(self.base[:, var] == self.base[:1, var]):
            raise ValueError("a theta-dependent entry changes with the regime: not an affine layout of this form")
        self.nparam, self.nregimes = nparam, nregimes

    def evaluate(self, theta, regime=None):
        """The device kernel's arithmetic (mpc_device.hip::k_affine) in numpy, per instance."""
        theta = np.atleast_2d(theta)
        B = theta.shape[0]
        reg = np.zeros(B, int) if regime is None else np.clip(np.asarray(regime), 0, self.nregimes - 1)
        out = np.empty((B, self.base.shape[1]))
        for b in range(B):
            bv = self.base[reg[b]]
            for i in range(out.shape[1]):
                v, anyt = 0.0, False
                for t in range(self.T):
                    k = self.idx[i, t]
                    if k >= 0:
                        term = self.coef[i, t] * theta[b, k]
                        v = v + term if anyt else term
                        anyt = True
                out[b, i] = bv[i] if not anyt else (bv[i] + v if bv[i] != 0.0 else v)
        s0, s1 = self.seglen[0], self.seglen[0] + self.seglen[1]
        return out[:, :s0], out[:, s0:s1], out[:, s1:]


def lateral_builder(layout, N):
    """(build(theta, regime) -> (q, l, u), nparam, nregimes, (P, A)) of a lateral layout.
    vanilla (Control/MPC/mpc_kinematics.py:148-191 with the lateral Ad / Bd, cfg 2):
      theta = (x0 (4), Xr stage-major ((N+1) x 4)), one regime;
    slack (vehicle_lateral_mpc_slack_increment.py:48-115 and :201-229, cfg 1 / 3 / 4):
      theta = (x~0 (5), xr (4)), regime 0 (i <= 400 or i > 900) / 1 (400 < i <= 900, :163-167)."""
    from . import mpc
    if layout == "vanilla":
        def build(theta, regime):
            x0, Xr = theta[:4], theta[4:].reshape(N + 1, 4).T
            P, q, A, l, u = mpc.vanilla_qp(mpc.LATERAL_AD, mpc.LATERAL_BD, np.zeros(4), x0, Xr, mpc.VANILLA_Q,
                                           mpc.VANILLA_Q, mpc.VANILLA_R, N, mpc.VANILLA_XMIN, -mpc.VANILLA_XMIN,
                                           -mpc.VANILLA_UMAX, mpc.VANILLA_UMAX)
            return q, l, u
        nparam, nreg = 4 + 4 * (N + 1), 1
        P, _, A, _, _ = mpc.vanilla_qp(mpc.LATERAL_AD, mpc.LATERAL_BD, np.zeros(4), np.zeros(4), np.zeros((4, N + 1)),
                                       mpc.VANILLA_Q, mpc.VANILLA_Q, mpc.VANILLA_R, N, mpc.VANILLA_XMIN,
                                       -mpc.VANILLA_XMIN, -mpc.VANILLA_UMAX, mpc.VANILLA_UMAX)
    elif layout == "slack":
        def build(theta, regime):
            _, q, _, l, u = mpc.slack_qp(N, theta[:5], xr=theta[5:9], regime=regime)
            return q, l, u
        nparam, nreg = 9, 2
        P, _, A, _, _ = mpc.slack_qp(N, np.zeros(5))
    else:
        raise ValueError(layout)
    return build, nparam, nreg, (P, A)


class LateralAssembler:
    """F1 for the lateral layouts on the device: q, l, u of B instances from their parameters
    theta = (x0, xr) and bound regimes (mpcqp_affine_apply_device); P and A are the layout's
    own, the same for every instance (DeviceBatch.setup_solve with 1-D Px / Ax: the shared-
    matrix mode).  Replaces the reference's per-step rebuild of the whole QP in Python
    (vehicle_lateral_mpc_slack_increment.py:132-229, ~6.5 ms per step)."""

    def __init__(self, layout, N=20, device=0):
        L = _bind()
        build, nparam, nreg, (P, A) = lateral_builder(layout, N)
        self.map = AffineMap(build, nparam, nreg)
        self.P, self.A = P, A
        self.n, self.m = P.shape[0], A.shape[0]
        self.nparam, self.nregimes = nparam, nreg
        m = self.map
        seg = np.ascontiguousarray(np.array(m.seglen, np.int32))
        self._keep = (seg, m.base, np.ascontiguousarray(m.idx), np.ascontiguousarray(m.coef))
        h = C.c_void_p()
        _check(L.mpcqp_affine_create(len(m.seglen), _np_ptr(seg), m.nregimes, m.T, _np_ptr(m.base),
                                     _np_ptr(self._keep[2]), _np_ptr(self._keep[3]), int(device), C.byref(h)),
               "affine_create")
        self._h = h.value
        self._free = L.mpcqp_affine_free
        self.device = int(device)

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            self._free(h)

    def matrices(self):
        """(Px, Ax): the layout's P (upper triangle) and A values in CSC order (host numpy)."""
        import scipy.sparse as sp
        P = sp.triu(sp.csc_matrix(self.P), format="csc")
        P.sort_indices()
        A = sp.csc_matrix(self.A)
        A.sort_indices()
        return P.data.copy(), A.data.copy()

    def assemble(self, theta, regime=None, out=None, stream=None):
        """theta (B, nparam) float64 and regime (B,) int32 device tensors -> (q, l, u) device
        tensors (into `out` when given)."""
        import torch
        L = _bind()
        B = theta.shape[0]
        if theta.dim() != 2 or theta.shape[1] < self.nparam or theta.stride(1) != 1:
            raise ValueError(f"theta must be (B, >= {self.nparam}) with a contiguous last axis")
        if regime is not None and (regime.dtype != torch.int32 or regime.shape[0] != B):
            raise ValueError("regime must be an int32 (B,) tensor")
        if out is None:
            kw = dict(dtype=torch.float64, device=theta.device)
            out = (torch.empty((B, self.n), **kw), torch.empty((B, self.m), **kw), torch.empty((B, self.m), **kw))
        st = stream if stream is not None else _stream(torch, theta.device)
        _check(L.mpcqp_affine_apply_device(self._h, B, _p(theta), theta.stride(0),
                                           None if regime is None else _p(regime), *(_p(t) for t in out), st),
               "affine_apply")
        return out


def reference_search(path_x, path_y, pred, dt):
    """reference_search (mpc_dynamics.py:44-90) per vehicle: pred (B, N+1, nxa) device tensor
    of predicted augmented states -> Xr (B, 6, N+1)."""
    import torch
    L = _bind()
    B, N1, nxa = pred.shape
    Xr = torch.empty((B, 6, N1), dtype=torch.float64, device=pred.device)
    _check(L.mpcqp_reference_search_device(B, N1 - 1, nxa, path_x.numel(), _p(path_x), _p(path_y), _p(pred),
                                           float(dt), _p(Xr), pred.device.index or 0, _stream(torch, pred.device)),
           "reference_search")
    return Xr


def warm_shift(N, nxa, nu, x, y=None):
    """Shift an incremental-layout solution (x (B, n), y (B, m) device tensors) one stage
    forward for warm-starting the next step (mpcqp_incr_warm_shift_device)."""
    import torch
    L = _bind()
    xs = torch.empty_like(x)
    ys = None if y is None else torch.empty_like(y)
    _check(L.mpcqp_incr_warm_shift_device(x.shape[0], int(N), int(nxa), int(nu), _p(x),
                                          None if y is None else _p(y), _p(xs), None if y is None else _p(ys),
                                          x.device.index or 0, _stream(torch, x.device)), "incr_warm_shift")
    return xs, ys


class DynamicMPC:
    """B copies of mpc_dynamics.main's closed loop (:437-617), every step on the device.

    State per vehicle: x~ = (X, Y, yaw, vx, vy, r, steer, accel), the predicted
    horizon pred_x~ (N+1 stages) and pred_du.  ``step()`` = reference search ->
    linearisation of every predicted stage -> mpc_increment's QP -> batched OSQP
    solve (settings of :393: polish off, warm_start off) -> plant step and shift.

    ``warm_start=True`` (an extension; the reference solves every step cold) starts
    each solve from the previous step's solution shifted one stage (warm_shift)."""

    Q = np.diag([100.0, 100.0, 100.0, 50.0, 50.0, 50.0])          # :456-458
    QN = np.diag([1000.0, 1000.0, 1000.0, 500.0, 500.0, 500.0])
    R = np.diag([50.0, 50.0])
    DUMIN = np.array([-np.deg2rad(2.0), -0.5])                      # :461-464
    XMIN_T = np.array([-np.inf, -np.inf, -2 * np.pi, -100., -30., -0.5 * np.pi, -np.deg2rad(15), -3.])
    XMAX_T = np.array([np.inf, np.inf, 2 * np.pi, 100., 30., 0.5 * np.pi, np.deg2rad(15), 1.])

    def __init__(self, x0, u0, path_x, path_y, N=30, veh: Vehicle | None = None, device=0, **solver_settings):
        import torch
        self.torch = torch
        self.dev = torch.device("cuda", device)
        self.veh = veh or Vehicle()
        self.N = int(N)
        x0 = np.atleast_2d(np.asarray(x0, np.float64)); u0 = np.atleast_2d(np.asarray(u0, np.float64))
        self.B = x0.shape[0]
        self.layout = IncrementalLayout(self.N, self.Q, self.QN, self.R, self.XMIN_T, self.XMAX_T, self.DUMIN,
                                        -self.DUMIN, device=device)
        P, A, _, _ = self.layout.pattern()
        settings = dict(verbose=False, polish=False, warm_start=False)   # mpc_dynamics.py:393
        settings.update(solver_settings)
        settings.pop("verbose", None)
        self.warm = bool(settings.pop("warm_start"))
        self.have_sol = False
        self.solver = DeviceBatch(P, A, self.B, device=device, **settings)
        kw = dict(dtype=torch.float64, device=self.dev)
        self.Px = torch.from_numpy(np.tile(P.data, (self.B, 1))).to(**kw).contiguous()
        self.path_x = torch.as_tensor(np.asarray(path_x, np.float64), **kw).contiguous()
        self.path_y = torch.as_tensor(np.asarray(path_y, np.float64), **kw).contiguous()
        self.xt = torch.from_numpy(np.concatenate([x0, u0], axis=1)).to(**kw).contiguous()
        n, m = self.layout.n, self.layout.m
        self.sol = torch.empty((self.B, n), **kw)
        self.y = torch.empty((self.B, m), **kw)
        self.status = torch.empty(self.B, dtype=torch.int32, device=self.dev)
        self.iters = torch.empty(self.B, dtype=torch.int32, device=self.dev)
        self.pdu = torch.zeros((self.B, self.N + 1, 2), **kw)
        # every kernel of a step runs on this stream, in order; a null (legacy default)
        # torch stream would be passed as NULL, which the solver's C ABI reads as "the
        # handle's own stream" -- unordered with torch's kernels
        self.stream = torch.cuda.Stream(self.dev)
        self.stream.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(self.stream):
            self.pred = self._initial_rollout()
        torch.cuda.current_stream(self.dev).wait_stream(self.stream)

    def _initial_rollout(self):
        """Initial guess (:513-522): roll the linearised model forward with zero increments."""
        torch = self.torch
        pred = torch.empty((self.B, self.N + 1, 8), dtype=torch.float64, device=self.dev)
        pred[:, 0] = self.xt
        xk = self.xt.clone()
        for i in range(self.N):
            Ad, Bd, gd = linearise(self.veh, xk[:, :6].contiguous(), xk[:, 6:].contiguous(), self.dev.index or 0)
            x1 = torch.einsum("bij,bj->bi", Ad, xk[:, :6]) + torch.einsum("bij,bj->bi", Bd, xk[:, 6:]) + gd
            xk = torch.cat([x1, xk[:, 6:] + self.pdu[:, i]], dim=1)
            pred[:, i + 1] = xk
        return pred

    def step(self):
        """One receding-horizon step for every vehicle; returns (status, iters) device tensors.
        Asynchronous: ordered after the caller's current stream, and the caller's stream
        is ordered after the step."""
        torch = self.torch
        caller = torch.cuda.current_stream(self.dev)
        self.stream.wait_stream(caller)
        with torch.cuda.stream(self.stream):
            out = self._step()
        caller.wait_stream(self.stream)
        return out

    def _step(self):
        L = _bind()
        torch = self.torch
        Xr = reference_search(self.path_x, self.path_y, self.pred, self.veh.dt)
        Ad, Bd, gd = linearise(self.veh, self.pred[:, :self.N, :6], self.pred[:, :self.N, 6:], self.dev.index or 0)
        Ax, q, l, u = self.layout.assemble(Ad, Bd, gd, self.xt, Xr)
        st = _stream(torch, self.dev)  # self.stream
        self.solver.setup(self.Px, Ax, q, l, u, stream=st)
        if self.warm and self.have_sol:
            xs, ys = warm_shift(self.N, 8, 2, self.sol, self.y)
            self.solver.warm_start(xs, ys, stream=st)
        self.solver.solve(self.sol, self.y, self.status, self.iters, stream=st)
        self.have_sol = True
        _check(L.mpcqp_incr_shift_device(self.layout._h, C.byref(self.veh), self.B, _p(self.sol), _p(Ad), _p(Bd),
                                         _p(gd), _p(self.xt), _p(self.pred), _p(self.pdu),
                                         _stream(torch, self.dev)), "incr_shift")
        self.last = dict(Ad=Ad, Bd=Bd, gd=gd, Xr=Xr, Ax=Ax, q=q, l=l, u=u)
        return self.status, self.iters
