// mpc_device.hip -- the MPC data path around the solver, on the device
// (SURVEY.md §8f rows F1-F3): everything the reference does in Python between two
// osqp solves of Control/MPC/mpc_dynamics.py:main, batched over B vehicles.
//
//   F2  k_linearise      Vehicle_Dynamics.get_dynamics_model   vehicle_models.py:52-340
//   F1  k_incr_assemble  mpc_increment's QP values             mpc_dynamics.py:281-389
//   F3  k_reference      reference_search / nearest_point       mpc_dynamics.py:30-90
//       k_incr_shift     plant step + horizon shift              mpc_dynamics.py:578-617
//                        (terminal state: update_dynamics_model  vehicle_models.py:343-477)
//
// One thread per (vehicle, stage) for the linearisation and per vehicle for the
// sequential parts (reference search walks the path, the shift reorders the
// horizon); one thread per (vehicle, A entry) for the assembly, which is a
// scatter of stage blocks into the shared CSC pattern.  All fp64.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>
#include <vector>

#include "../../include/mpcqp.h"
#include "kernels.h"

namespace mpcqp {

// ------------------------------------------------------------------- vehicle --
// Constants of Vehicle_Dynamics (vehicle_models.py:27-50) and of its lateral
// Pacejka tyre model (vehicle_models.py:114-132: B in 1/rad, C, D per axle),
// derived once on the host with the reference's own formulas.
struct VehicleK {
    double m, lf, lr, Iz, dt, cda;  // cda = roh * C_d * A_f
    double roll;                    // C_roll * m * 9.81
    double Bf, Cf, Df, Br, Cr, Dr;
};

static VehicleK vehicle_constants(const mpcqp_vehicle& v) {
    VehicleK k;
    k.m = v.m; k.lf = v.l_f; k.lr = v.l_r; k.dt = v.dt;
    k.Iz = 1.0 / 12 * v.m * (v.width * v.width + v.length * v.length);
    const double roh = 1.23;
    k.cda = roh * v.C_d * v.A_f;
    k.roll = v.C_roll * v.m * 9.81;
    const double a[8] = {-22.1, 1011, 1078, 1.82, 0.208, 0.000, -0.354, 0.707};
    const double wheelbase = v.l_f + v.l_r;
    const double pi = 3.141592653589793;
    for (int axle = 0; axle < 2; ++axle) {
        const double Fz = 9.81 * (v.m * (axle == 0 ? v.l_r : v.l_f) / wheelbase) * 0.001;
        const double C = 1.30;
        const double D = a[0] * Fz * Fz + a[1] * Fz;
        const double BCD = a[2] * std::sin(a[3] * std::atan(a[4] * Fz));
        const double B = BCD / (C * D) * 180 / pi;
        if (axle == 0) { k.Bf = B; k.Cf = C; k.Df = D; }
        else { k.Br = B; k.Cr = C; k.Dr = D; }
    }
    return k;
}

__device__ __forceinline__ double sgn(double v) { return v > 0.0 ? 1.0 : (v < 0.0 ? -1.0 : 0.0); }

// low-speed guard of get_dynamics_model / update_dynamics_model (vehicle_models.py:143-159),
// on copies: 0 <= vx < 0.5 or -0.5 < vx < 0 -> vy = r = steer = 0 and |vx| >= 0.3
__device__ __forceinline__ void low_speed_guard(double* x, double* u) {
    const double vx = x[3];
    if (vx >= 0.0 && vx < 0.5) {
        x[4] = 0.0; x[5] = 0.0; u[0] = 0.0;
        if (vx < 0.3) x[3] = 0.3;
    }
    if (x[3] > -0.5 && x[3] < 0.0) {
        x[4] = 0.0; x[5] = 0.0; u[0] = 0.0;
        if (x[3] > -0.3) x[3] = -0.3;
    }
}

// f(x, u) of the dynamic bicycle model (vehicle_models.py:238-245 / 470-475), plus the
// tyre quantities the Jacobian needs
struct Tyre {
    double af, ar, Fyf, Fyr, Fx;
};
__device__ __forceinline__ Tyre tyre_forces(const VehicleK& k, const double* x, const double* u) {
    Tyre t;
    const double vx = x[3], vy = x[4], r = x[5], st = u[0], acc = u[1];
    t.af = -atan2(k.lf * r + vy, vx) + st;
    t.ar = -atan2(-k.lr * r + vy, vx);
    t.Fyf = k.Df * sin(k.Cf * atan(k.Bf * t.af));
    t.Fyr = k.Dr * sin(k.Cr * atan(k.Br * t.ar));
    const double R_roll = k.roll * sgn(vx);
    const double F_aero = 0.5 * k.cda * vx * vx * sgn(vx);
    t.Fx = k.m * acc - F_aero - R_roll;
    return t;
}
__device__ __forceinline__ void dynamics(const VehicleK& k, const double* x, const double* u, const Tyre& t,
                                         double* f) {
    const double yaw = x[2], vx = x[3], vy = x[4], r = x[5], st = u[0];
    const double cy = cos(yaw), sy = sin(yaw), cs = cos(st), ss = sin(st);
    f[0] = vx * cy - vy * sy;
    f[1] = vy * cy + vx * sy;
    f[2] = r;
    f[3] = 1. / k.m * (t.Fx * cs - t.Fyf * ss + k.m * vy * r);
    f[4] = 1. / k.m * (t.Fx * ss + t.Fyr + t.Fyf * cs - k.m * vx * r);
    f[5] = 1. / k.Iz * (t.Fx * k.lf * ss + t.Fyf * k.lf * cs - t.Fyr * k.lr);
}

// get_dynamics_model for one (x, u): Ad = I + dt Ac, Bd = dt Bc, gd = dt (f - Ac x - Bc u)
__device__ void linearise_one(const VehicleK& k, const double* xin, const double* uin, double* __restrict__ Ad,
                              double* __restrict__ Bd, double* __restrict__ gd) {
    double x[6], u[2];
    for (int i = 0; i < 6; ++i) x[i] = xin[i];
    u[0] = uin[0]; u[1] = uin[1];
    low_speed_guard(x, u);
    const Tyre t = tyre_forces(k, x, u);
    double f[6];
    dynamics(k, x, u, t, f);
    const double yaw = x[2], vx = x[3], vy = x[4], r = x[5], st = u[0];
    const double m = k.m, Iz = k.Iz, lf = k.lf, lr = k.lr;
    const double cy = cos(yaw), sy = sin(yaw), cs = cos(st), ss = sin(st);
    // :251-270 tyre-force derivatives
    const double dFxf_dvx = -k.cda * vx;
    const double dFxf_daccel = m;
    const double kf = (k.Bf * k.Cf * k.Df * cos(k.Cf * atan(k.Bf * t.af))) / (1 + k.Bf * k.Bf * t.af * t.af);
    const double kr = (k.Br * k.Cr * k.Dr * cos(k.Cr * atan(k.Br * t.ar))) / (1 + k.Br * k.Br * t.ar * t.ar);
    const double af_num = lf * r + vy, ar_num = -lr * r + vy;
    const double nf = af_num * af_num + vx * vx, nr = ar_num * ar_num + vx * vx;
    const double dFyf_dvx = kf * af_num / nf;
    const double dFyf_dvy = kf * (-vx / nf);
    const double dFyf_dr = kf * (-lf * vx) / nf;
    const double dFyf_dst = kf;
    const double dFyr_dvx = kr * ar_num / nr;
    const double dFyr_dvy = kr * (-vx) / nr;
    const double dFyr_dr = kr * (lr * vx) / nr;
    // :273-292 Jacobians
    double Ac[36] = {0.0}, Bc[12] = {0.0};
    Ac[0 * 6 + 2] = -vx * sy - vy * cy; Ac[0 * 6 + 3] = cy; Ac[0 * 6 + 4] = -sy;
    Ac[1 * 6 + 2] = -vy * sy + vx * cy; Ac[1 * 6 + 3] = sy; Ac[1 * 6 + 4] = cy;
    Ac[2 * 6 + 5] = 1.;
    Ac[3 * 6 + 3] = 1 / m * (dFxf_dvx * cs - dFyf_dvx * ss);
    Ac[3 * 6 + 4] = 1 / m * (-dFyf_dvy * ss + m * r);
    Ac[3 * 6 + 5] = 1 / m * (-dFyf_dr * ss + m * vy);
    Ac[4 * 6 + 3] = 1 / m * (dFxf_dvx * ss + dFyr_dvx + dFyf_dvx * cs - m * r);
    Ac[4 * 6 + 4] = 1 / m * (dFyr_dvy + dFyf_dvy * cs);
    Ac[4 * 6 + 5] = 1 / m * (dFyr_dr + dFyf_dr * cs - m * vx);
    Ac[5 * 6 + 3] = 1 / Iz * (dFxf_dvx * lf * ss + dFyf_dvx * lf * cs - dFyr_dvx * lr);
    Ac[5 * 6 + 4] = 1 / Iz * (dFyf_dvy * lf * cs - dFyr_dvy * lr);
    Ac[5 * 6 + 5] = 1 / Iz * (dFyf_dr * lf * cs - dFyr_dr * lr);
    Bc[3 * 2 + 0] = 1 / m * (-t.Fx * ss - dFyf_dst * ss - t.Fyf * cs);
    Bc[3 * 2 + 1] = 1 / m * (dFxf_daccel * cs);
    Bc[4 * 2 + 0] = 1 / m * (t.Fx * cs + dFyf_dst * cs - t.Fyf * ss);
    Bc[4 * 2 + 1] = 1 / m * (dFxf_daccel * ss);
    Bc[5 * 2 + 0] = 1 / Iz * (t.Fx * lf * cs + dFyf_dst * lf * cs - t.Fyf * lf * ss);
    Bc[5 * 2 + 1] = 1 / Iz * (dFxf_daccel * lf * ss);
    // :294, :318-324
    for (int i = 0; i < 6; ++i) {
        double ax = 0.0;
        for (int j = 0; j < 6; ++j) ax += Ac[i * 6 + j] * x[j];
        const double bu = Bc[i * 2 + 0] * u[0] + Bc[i * 2 + 1] * u[1];
        gd[i] = (f[i] - ax - bu) * k.dt;
        for (int j = 0; j < 6; ++j) Ad[i * 6 + j] = (i == j ? 1.0 : 0.0) + Ac[i * 6 + j] * k.dt;
        Bd[i * 2 + 0] = Bc[i * 2 + 0] * k.dt;
        Bd[i * 2 + 1] = Bc[i * 2 + 1] * k.dt;
    }
}

__global__ __launch_bounds__(256) void k_linearise(VehicleK k, long B, int N, const double* __restrict__ x, long x_sb,
                                                   long x_sk, const double* __restrict__ u, long u_sb, long u_sk,
                                                   double* __restrict__ Ad, double* __restrict__ Bd,
                                                   double* __restrict__ gd) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= B * N) return;
    const long b = t / N, s = t - b * N;
    linearise_one(k, x + b * x_sb + s * x_sk, u + b * u_sb + s * u_sk, Ad + t * 36, Bd + t * 12, gd + t * 6);
}

// update_dynamics_model (vehicle_models.py:343-477): one explicit-Euler step of the
// nonlinear model from the guarded state
__device__ void euler_step(const VehicleK& k, const double* xin, const double* uin, double* xn) {
    double x[6], u[2];
    for (int i = 0; i < 6; ++i) x[i] = xin[i];
    u[0] = uin[0]; u[1] = uin[1];
    low_speed_guard(x, u);
    const Tyre t = tyre_forces(k, x, u);
    double f[6];
    dynamics(k, x, u, t, f);
    for (int i = 0; i < 6; ++i) xn[i] = x[i] + f[i] * k.dt;
}

// ------------------------------------------------------- incremental QP layout --
// The QP of mpc_increment (mpc_dynamics.py:281-389) for nxa = nx + nu augmented
// states:  variables (x~_0 .. x~_N, du_0 .. du_{N-1}),
//   A = [ Aeq ; I ],  Aeq = [ -I + subdiag(A~_k) | B~_k shifted one block down ],
//   A~_k = [[Ad_k, Bd_k], [0, I]],  B~_k = [Bd_k; I].
// The pattern keeps every STRUCTURAL nonzero of Ad / Bd (masks), so it does not
// change when a value happens to be 0 (the reference's scipy pattern does; the
// QP is the same -- an explicit zero contributes nothing to OSQP's arithmetic).
// Ax source codes: >= 0 -> Ad entry (stage * nx*nx + i*nx + j); -1 - c -> Bd entry
// c = stage * nx*nu + i*nu + j; kConst -> the template value.
constexpr int kConstSrc = INT32_MIN;

struct IncrLayout {
    int N = 0, nx = 0, nu = 0, nxa = 0, n = 0, m = 0, dev = 0;
    std::vector<int> Pp, Pi, Ap, Ai, asrc;
    std::vector<double> Px, Atpl, ltpl, utpl, Qt, QNt;  // Qt / QNt: (Q C)' rows i < nx (nx x nx, [i][j] = Q[j][i])
    int* d_asrc = nullptr;
    double *d_Atpl = nullptr, *d_ltpl = nullptr, *d_utpl = nullptr, *d_Qt = nullptr;
};

struct IncrK {  // what the device kernels need (by value)
    int N, nx, nu, nxa, n, m, nnzA;
    const int* asrc;
    const double *Atpl, *ltpl, *utpl, *Qt;  // Qt: [2][nx*nx] (stage weights, terminal weights)
};

__global__ __launch_bounds__(256) void k_incr_assemble_A(IncrK L, long B, const double* __restrict__ Ad,
                                                         const double* __restrict__ Bd, double* __restrict__ Ax) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= B * L.nnzA) return;
    const long b = t / L.nnzA;
    const int e = (int)(t - b * L.nnzA);
    const int s = L.asrc[e];
    double v;
    if (s == kConstSrc) v = L.Atpl[e];
    else if (s >= 0) v = Ad[b * (long)L.N * L.nx * L.nx + s];
    else v = Bd[b * (long)L.N * L.nx * L.nu + (-1 - s)];
    Ax[t] = v;
}

// q, l, u of one vehicle per thread
__global__ __launch_bounds__(128) void k_incr_assemble_vec(IncrK L, long B, const double* __restrict__ gd,
                                                           const double* __restrict__ xt0,
                                                           const double* __restrict__ Xr, double* __restrict__ q,
                                                           double* __restrict__ l, double* __restrict__ u) {
    const long b = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const int N = L.N, nx = L.nx, nxa = L.nxa, n = L.n, m = L.m;
    // q = [ -(Q C)' Xr_k  (k < N) ; -(QN C)' Xr_N ; 0 ]   (:313-319)
    double* qb = q + b * n;
    const double* Xb = Xr + b * (long)nx * (N + 1);  // Xr[j][k] at j*(N+1)+k
    for (int k = 0; k <= N; ++k) {
        const double* W = L.Qt + (k == N ? nx * nx : 0);
        for (int i = 0; i < nxa; ++i) {
            double acc = 0.0;
            if (i < nx)
                for (int j = 0; j < nx; ++j) acc += W[i * nx + j] * Xb[j * (N + 1) + k];
            qb[k * nxa + i] = -acc;
        }
    }
    for (int i = (N + 1) * nxa; i < n; ++i) qb[i] = 0.0;
    // leq = ueq = [ -x~_0 ; -g~_k ],  g~_k = [gd_k; 0]   (:371-378); inequality rows: template
    double* lb = l + b * m;
    double* ub = u + b * m;
    for (int i = 0; i < nxa; ++i) lb[i] = ub[i] = -xt0[b * nxa + i];
    const double* gb = gd + b * (long)N * nx;
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < nxa; ++i) {
            const double v = i < nx ? -gb[k * nx + i] : -0.0;
            lb[(k + 1) * nxa + i] = ub[(k + 1) * nxa + i] = v;
        }
    for (int r = (N + 1) * nxa; r < m; ++r) {
        lb[r] = L.ltpl[r];
        ub[r] = L.utpl[r];
    }
}

// ---------------------------------------------------------- receding horizon --
// reference_search (mpc_dynamics.py:44-90) with nearest_point (:30-41, look_ind = 1):
// Xr[:, i] = (path point, yaw 0, vx 10, vy 0, r 0) where the path index walks forward
// while the travelled distance sum |vx_i| dt exceeds the path length covered.
// pred: (B, N+1, nxa) stage-major;  Xr: (B, 6, N+1).
__global__ __launch_bounds__(128) void k_reference(long B, int N, int nxa, int np, const double* __restrict__ px,
                                                   const double* __restrict__ py, const double* __restrict__ pred,
                                                   double dt, double* __restrict__ Xr) {
    const long b = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const double* pb = pred + b * (long)(N + 1) * nxa;
    const double X0 = pb[0], Y0 = pb[1];
    double min_d = INFINITY;
    int ind = -1;
    for (int i = np - 1; i >= 0; --i) {  // reversed(range(len(path_x))), strict <
        const double d = sqrt((px[i] - X0) * (px[i] - X0) + (py[i] - Y0) * (py[i] - Y0));
        if (d < min_d) { min_d = d; ind = i; }
    }
    // look_ind = 1.  The reference reads path[ind + 1] from here on and raises
    // IndexError once ind reaches the last point; the kernel holds the start of the
    // last segment (np - 2) instead.
    ind = min(ind + 1, np - 2);
    auto seg = [&](int i) {
        return sqrt((px[i + 1] - px[i]) * (px[i + 1] - px[i]) + (py[i + 1] - py[i]) * (py[i + 1] - py[i]));
    };
    double path_d = seg(ind), cumul = 0.0;
    double* Xb = Xr + b * 6L * (N + 1);
    for (int i = 0; i <= N; ++i) {
        cumul += fabs(pb[i * nxa + 3]) * dt;
        while (cumul >= path_d && ind + 1 < np - 1) {
            ind += 1;
            path_d += seg(ind);
        }
        const int ic = ind;
        Xb[0 * (N + 1) + i] = px[ic];
        Xb[1 * (N + 1) + i] = py[ic];
        Xb[2 * (N + 1) + i] = 0.0;
        Xb[3 * (N + 1) + i] = 10.0;
        Xb[4 * (N + 1) + i] = 0.0;
        Xb[5 * (N + 1) + i] = 0.0;
    }
}

// One-stage shift of a vector made of `groups` blocks of N+1 stages of width nxa followed
// by one block of N stages of width nu (x: groups 1, y: groups 2); element-parallel.
__global__ __launch_bounds__(256) void k_stage_shift(long total, int len, int N, int nxa, int nu, int groups,
                                                     const double* __restrict__ src, double* __restrict__ dst) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= total) return;
    const long b = e / len;
    const int i = (int)(e - b * len);
    const int stage_blk = (N + 1) * nxa, head = groups * stage_blk;
    int j;
    if (i < head) {
        const int g = i / stage_blk, r = i - g * stage_blk, k = r / nxa, c = r - k * nxa;
        j = g * stage_blk + min(k + 1, N) * nxa + c;
    } else {
        const int r = i - head, k = r / nu, c = r - k * nu;
        j = head + min(k + 1, N - 1) * nu + c;
    }
    dst[e] = src[b * len + j];
}

// plant step and horizon shift of mpc_dynamics.main (:578-617), per vehicle:
//   pred_x~[:, k] = sol[k nxa ..],  du[:, k] = sol[(N+1) nxa + k nu ..]  (mpc_increment :398-432)
//   u = u_past + du_0;  x_next = Ad_0 x + Bd_0 u + gd_0;  x~ = (x_next, u)
//   shift pred_x~ / du one stage; terminal state by one nonlinear Euler step from
//   (pred_x~[:nx, N], pred_x~[nx:, N-1]) (update_dynamics_model)
__global__ __launch_bounds__(128) void k_incr_shift(VehicleK vk, IncrK L, long B, const double* __restrict__ sol,
                                                    const double* __restrict__ Ad, const double* __restrict__ Bd,
                                                    const double* __restrict__ gd, double* __restrict__ xt,
                                                    double* __restrict__ pred, double* __restrict__ pdu) {
    const long b = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const int N = L.N, nx = L.nx, nu = L.nu, nxa = L.nxa, n = L.n;
    const double* s = sol + b * n;
    double* pb = pred + b * (long)(N + 1) * nxa;
    double* db = pdu + b * (long)(N + 1) * nu;
    const double* A0 = Ad + b * (long)N * nx * nx;  // stage 0
    const double* B0 = Bd + b * (long)N * nx * nu;
    const double* g0 = gd + b * (long)N * nx;
    double* xb = xt + b * nxa;
    // plant step (:581-586)
    double xnext[8], uu[8];
    for (int j = 0; j < nu; ++j) uu[j] = xb[nx + j] + s[(N + 1) * nxa + j];
    for (int i = 0; i < nx; ++i) {
        double acc = 0.0;
        for (int j = 0; j < nx; ++j) acc += A0[i * nx + j] * xb[j];
        double bu = 0.0;
        for (int j = 0; j < nu; ++j) bu += B0[i * nu + j] * uu[j];
        xnext[i] = (acc + bu) + g0[i];
    }
    for (int i = 0; i < nx; ++i) xb[i] = xnext[i];
    for (int j = 0; j < nu; ++j) xb[nx + j] = uu[j];
    // shift (:589-610) from the solution (the reference's temp copies are the solution)
    for (int i = 0; i < nxa; ++i) pb[i] = xb[i];
    for (int j = 0; j < nu; ++j) db[j] = s[(N + 1) * nxa + 1 * nu + j];
    for (int k = 1; k <= N - 2; ++k) {
        for (int i = 0; i < nxa; ++i) pb[k * nxa + i] = s[(k + 1) * nxa + i];
        for (int j = 0; j < nu; ++j) db[k * nu + j] = s[(N + 1) * nxa + (k + 1) * nu + j];
    }
    for (int i = 0; i < nxa; ++i) pb[(N - 1) * nxa + i] = s[N * nxa + i];
    for (int j = 0; j < nu; ++j) db[(N - 1) * nu + j] = s[(N + 1) * nxa + (N - 1) * nu + j];
    // terminal state (:604-608): Euler step of (x_N, u_{N-1}) of the solution
    double xN[6], uN[2], xe[6];
    for (int i = 0; i < 6; ++i) xN[i] = s[N * nxa + i];
    for (int j = 0; j < 2; ++j) uN[j] = s[(N - 1) * nxa + nx + j];
    euler_step(vk, xN, uN, xe);
    for (int i = 0; i < nx; ++i) pb[N * nxa + i] = xe[i];
    for (int j = 0; j < nu; ++j) pb[N * nxa + nx + j] = pb[(N - 1) * nxa + nx + j];
    for (int j = 0; j < nu; ++j) db[N * nu + j] = db[(N - 1) * nu + j];
}

// ---- F1 for the LTI (lateral) layouts: affine vector assembly ----
// vehicle_lateral_mpc_slack_increment.py:32-121 / its loop :201-229 and
// Control/MPC/mpc_kinematics.py:148-191 rebuild P, q, A, l, u every step although with the
// fixed lateral model only q (from xr), the initial-state rows of l = u (from x0) and the
// bound regime's inequality rows change.  Every entry of the concatenated (q, l, u) is an
// affine function of the instance's parameters theta = (x0, xr), with a base vector per
// bound regime:  v_i = base[regime][i] + sum_t coef[i][t] theta[idx[i][t]].  One thread per
// (instance, entry), consecutive threads on consecutive entries (coalesced stores).
struct AffineK {
    int L, R, T, seg0, seg1;  // entries, regimes, terms per entry, segment starts (q | l | u)
    const double *base, *coef;
    const int* idx;
};

__global__ __launch_bounds__(256) void k_affine(AffineK a, long B, const double* __restrict__ theta, int tstride,
                                                const int* __restrict__ regime, double* __restrict__ o0,
                                                double* __restrict__ o1, double* __restrict__ o2) {
    const long g = (long)blockIdx.x * 256 + threadIdx.x;
    if (g >= B * a.L) return;
    const long b = g / a.L;
    const int i = (int)(g - b * a.L);
    int r = regime ? regime[b] : 0;
    r = r < 0 ? 0 : (r >= a.R ? a.R - 1 : r);
    const double bv = a.base[(long)r * a.L + i];
    // the terms first, the base added only where it is nonzero: an entry the builder forms
    // as a product alone (q = -Q xr, l = u = -x0) is that product, bit for bit
    double v = 0.0;
    bool any = false;
    for (int t = 0; t < a.T; ++t) {
        const int k = a.idx[i * a.T + t];
        if (k >= 0) {
            const double term = a.coef[i * a.T + t] * theta[b * tstride + k];
            v = any ? v + term : term;
            any = true;
        }
    }
    v = !any ? bv : (bv != 0.0 ? bv + v : v);
    if (i < a.seg0) o0[b * a.seg0 + i] = v;
    else if (i < a.seg1) o1[b * (a.seg1 - a.seg0) + (i - a.seg0)] = v;
    else o2[b * (a.L - a.seg1) + (i - a.seg1)] = v;
}

}  // namespace mpcqp

using namespace mpcqp;

struct mpcqp_incr_layout : IncrLayout {};

struct mpcqp_affine {
    int dev = 0, L = 0, R = 0, T = 0, seg0 = 0, seg1 = 0, nparam = 0;
    double *d_base = nullptr, *d_coef = nullptr;
    int* d_idx = nullptr;
};

namespace {

#define MHIPCHK(expr)                                                                         \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return set_error(MPCQP_EDEVICE, "%s failed: %s", #expr, hipGetErrorString(e_));   \
    } while (0)

template <class T>
int upload(const std::vector<T>& v, T** d) {
    MHIPCHK(hipMalloc((void**)d, sizeof(T) * std::max<size_t>(v.size(), 1)));
    if (!v.empty()) MHIPCHK(hipMemcpy(*d, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice));
    return 0;
}

int ensure_device(IncrLayout& L) {
    if (L.d_asrc) return 0;
    MHIPCHK(hipSetDevice(L.dev));
    if (int e = upload(L.asrc, &L.d_asrc)) return e;
    if (int e = upload(L.Atpl, &L.d_Atpl)) return e;
    if (int e = upload(L.ltpl, &L.d_ltpl)) return e;
    if (int e = upload(L.utpl, &L.d_utpl)) return e;
    if (int e = upload(L.Qt, &L.d_Qt)) return e;
    return 0;
}

IncrK incr_k(const IncrLayout& L) {
    IncrK k;
    k.N = L.N; k.nx = L.nx; k.nu = L.nu; k.nxa = L.nxa; k.n = L.n; k.m = L.m; k.nnzA = (int)L.Ai.size();
    k.asrc = L.d_asrc; k.Atpl = L.d_Atpl; k.ltpl = L.d_ltpl; k.utpl = L.d_utpl; k.Qt = L.d_Qt;
    return k;
}

unsigned grid_of(long count, int block) { return (unsigned)((count + block - 1) / block); }

}  // namespace

extern "C" {

int mpcqp_linearise_device(const mpcqp_vehicle* veh, int64_t B, int32_t N, const double* dx, int64_t x_sb,
                           int64_t x_sk, const double* du, int64_t u_sb, int64_t u_sk, double* dAd, double* dBd,
                           double* dgd, int32_t device, void* stream) {
    if (!veh || !dx || !du || !dAd || !dBd || !dgd || B < 0 || N < 1)
        return set_error(MPCQP_EINVAL, "linearise: bad arguments");
    if (B == 0) return 0;
    MHIPCHK(hipSetDevice(device));
    const VehicleK k = vehicle_constants(*veh);
    hipLaunchKernelGGL(k_linearise, dim3(grid_of(B * N, 256)), dim3(256), 0, (hipStream_t)stream, k, (long)B, (int)N,
                       dx, (long)x_sb, (long)x_sk, du, (long)u_sb, (long)u_sk, dAd, dBd, dgd);
    MHIPCHK(hipGetLastError());
    return 0;
}

int mpcqp_incr_layout_create(int32_t N, int32_t nx, int32_t nu, const double* Q, const double* QN, const double* R,
                             const double* xmin_t, const double* xmax_t, const double* dumin, const double* dumax,
                             const uint8_t* maskA, const uint8_t* maskB, int32_t device, mpcqp_incr_layout** out) {
    if (!out || !Q || !QN || !R || !xmin_t || !xmax_t || !dumin || !dumax || !maskA || !maskB)
        return set_error(MPCQP_EINVAL, "incr_layout_create: NULL argument");
    if (N < 2 || nx < 1 || nu < 1 || nx > 6 || nu > 2)
        return set_error(MPCQP_EUNSUPPORTED, "incr_layout_create: need N >= 2, 1 <= nx <= 6, 1 <= nu <= 2");
    for (int i = 0; i < nx + nu; ++i)
        if (!(xmin_t[i] <= xmax_t[i])) return set_error(MPCQP_EINVAL, "incr_layout_create: xmin_t > xmax_t");
    for (int j = 0; j < nu; ++j)
        if (!(dumin[j] <= dumax[j])) return set_error(MPCQP_EINVAL, "incr_layout_create: dumin > dumax");
    *out = nullptr;
    auto L = std::make_unique<mpcqp_incr_layout>();
    const int nxa = nx + nu, n = (N + 1) * nxa + N * nu, m = (N + 1) * nxa + n;
    L->N = N; L->nx = nx; L->nu = nu; L->nxa = nxa; L->n = n; L->m = m; L->dev = device;
    const double INF = 1e30;  // the osqp wrapper clips +-inf to +-OSQP_INFTY
    // P = blockdiag(kron(I_N, C'QC), C'QN C, kron(I_N, R)), upper triangle, zeros dropped (:304-307)
    L->Pp.assign(n + 1, 0);
    for (int c = 0; c < n; ++c) {
        if (c < (N + 1) * nxa) {
            const int k = c / nxa, j = c % nxa;
            const double* W = k == N ? QN : Q;
            if (j < nx)
                for (int i = 0; i <= j; ++i) {
                    const double v = W[i * nx + j];
                    if (v != 0.0) { L->Pi.push_back(k * nxa + i); L->Px.push_back(v); }
                }
        } else {
            const int c0 = c - (N + 1) * nxa, k = c0 / nu, j = c0 % nu;
            for (int i = 0; i <= j; ++i) {
                const double v = R[i * nu + j];
                if (v != 0.0) { L->Pi.push_back((N + 1) * nxa + k * nu + i); L->Px.push_back(v); }
            }
        }
        L->Pp[c + 1] = (int)L->Pi.size();
    }
    // A by column (:336-369, :381-382)
    L->Ap.assign(n + 1, 0);
    auto push = [&](int row, int src, double tpl) {
        L->Ai.push_back(row); L->asrc.push_back(src); L->Atpl.push_back(tpl);
    };
    for (int c = 0; c < n; ++c) {
        if (c < (N + 1) * nxa) {
            const int k = c / nxa, j = c % nxa;
            push(k * nxa + j, kConstSrc, -1.0);  // -I
            if (k < N)                           // A~_k in rows of stage k+1
                for (int i = 0; i < nxa; ++i) {
                    const int row = (k + 1) * nxa + i;
                    if (i < nx && j < nx) {
                        if (maskA[i * nx + j]) push(row, k * nx * nx + i * nx + j, 0.0);
                    } else if (i < nx) {
                        if (maskB[i * nu + (j - nx)]) push(row, -1 - (k * nx * nu + i * nu + (j - nx)), 0.0);
                    } else if (i == j) {
                        push(row, kConstSrc, 1.0);
                    }
                }
        } else {
            const int c0 = c - (N + 1) * nxa, k = c0 / nu, j = c0 % nu;  // du_k: B~_k in rows of stage k+1
            for (int i = 0; i < nxa; ++i) {
                const int row = (k + 1) * nxa + i;
                if (i < nx) {
                    if (maskB[i * nu + j]) push(row, -1 - (k * nx * nu + i * nu + j), 0.0);
                } else if (i - nx == j) {
                    push(row, kConstSrc, 1.0);
                }
            }
        }
        push((N + 1) * nxa + c, kConstSrc, 1.0);  // A_ineq = I
        L->Ap[c + 1] = (int)L->Ai.size();
    }
    // inequality bounds (:383-384), clipped like the osqp wrapper
    L->ltpl.assign(m, 0.0); L->utpl.assign(m, 0.0);
    for (int k = 0; k <= N; ++k)
        for (int i = 0; i < nxa; ++i) {
            L->ltpl[(N + 1) * nxa + k * nxa + i] = std::max(xmin_t[i], -INF);
            L->utpl[(N + 1) * nxa + k * nxa + i] = std::min(xmax_t[i], INF);
        }
    for (int k = 0; k < N; ++k)
        for (int j = 0; j < nu; ++j) {
            L->ltpl[(N + 1) * nxa + (N + 1) * nxa + k * nu + j] = std::max(dumin[j], -INF);
            L->utpl[(N + 1) * nxa + (N + 1) * nxa + k * nu + j] = std::min(dumax[j], INF);
        }
    // (Q C)' restricted to its nx x nx nonzero block: [i][j] = W[j][i], stage and terminal
    L->Qt.assign(2 * nx * nx, 0.0);
    for (int i = 0; i < nx; ++i)
        for (int j = 0; j < nx; ++j) {
            L->Qt[i * nx + j] = Q[j * nx + i];
            L->Qt[nx * nx + i * nx + j] = QN[j * nx + i];
        }
    *out = L.release();  // device copies are made by the first assemble / shift (host-only use needs no GPU)
    return 0;
}

int mpcqp_incr_layout_dims(const mpcqp_incr_layout* L, int32_t* n, int32_t* m, int32_t* nnzP, int32_t* nnzA) {
    if (!L || !n || !m || !nnzP || !nnzA) return set_error(MPCQP_EINVAL, "incr_layout_dims: NULL argument");
    *n = L->n; *m = L->m; *nnzP = (int32_t)L->Pi.size(); *nnzA = (int32_t)L->Ai.size();
    return 0;
}

int mpcqp_incr_layout_pattern(const mpcqp_incr_layout* L, int32_t* Pp, int32_t* Pi, double* Px, int32_t* Ap,
                              int32_t* Ai, double* Ax_template, double* l_template, double* u_template) {
    if (!L) return set_error(MPCQP_EINVAL, "incr_layout_pattern: NULL layout");
    if (Pp) std::memcpy(Pp, L->Pp.data(), sizeof(int32_t) * L->Pp.size());
    if (Pi) std::memcpy(Pi, L->Pi.data(), sizeof(int32_t) * L->Pi.size());
    if (Px) std::memcpy(Px, L->Px.data(), sizeof(double) * L->Px.size());
    if (Ap) std::memcpy(Ap, L->Ap.data(), sizeof(int32_t) * L->Ap.size());
    if (Ai) std::memcpy(Ai, L->Ai.data(), sizeof(int32_t) * L->Ai.size());
    if (Ax_template) std::memcpy(Ax_template, L->Atpl.data(), sizeof(double) * L->Atpl.size());
    if (l_template) std::memcpy(l_template, L->ltpl.data(), sizeof(double) * L->ltpl.size());
    if (u_template) std::memcpy(u_template, L->utpl.data(), sizeof(double) * L->utpl.size());
    return 0;
}

int mpcqp_incr_assemble_device(const mpcqp_incr_layout* L, int64_t B, const double* dAd, const double* dBd,
                               const double* dgd, const double* dxt0, const double* dXr, double* dAx, double* dq,
                               double* dl, double* du, void* stream) {
    if (!L || !dAd || !dBd || !dgd || !dxt0 || !dXr || !dAx || !dq || !dl || !du || B < 0)
        return set_error(MPCQP_EINVAL, "incr_assemble: bad arguments");
    if (B == 0) return 0;
    if (int e = ensure_device(*const_cast<mpcqp_incr_layout*>(L))) return e;
    MHIPCHK(hipSetDevice(L->dev));
    const IncrK k = incr_k(*L);
    const long nA = (long)B * k.nnzA;
    hipLaunchKernelGGL(k_incr_assemble_A, dim3(grid_of(nA, 256)), dim3(256), 0, (hipStream_t)stream, k, (long)B,
                       dAd, dBd, dAx);
    hipLaunchKernelGGL(k_incr_assemble_vec, dim3(grid_of(B, 128)), dim3(128), 0, (hipStream_t)stream, k, (long)B,
                       dgd, dxt0, dXr, dq, dl, du);
    MHIPCHK(hipGetLastError());
    return 0;
}

int mpcqp_reference_search_device(int64_t B, int32_t N, int32_t nxa, int32_t npath, const double* dpath_x,
                                  const double* dpath_y, const double* dpred, double dt, double* dXr, int32_t device,
                                  void* stream) {
    if (!dpath_x || !dpath_y || !dpred || !dXr || B < 0 || N < 1 || nxa < 4 || npath < 2)
        return set_error(MPCQP_EINVAL, "reference_search: bad arguments");
    if (B == 0) return 0;
    MHIPCHK(hipSetDevice(device));
    hipLaunchKernelGGL(k_reference, dim3(grid_of(B, 128)), dim3(128), 0, (hipStream_t)stream, (long)B, (int)N,
                       (int)nxa, (int)npath, dpath_x, dpath_y, dpred, dt, dXr);
    MHIPCHK(hipGetLastError());
    return 0;
}

int mpcqp_incr_shift_device(const mpcqp_incr_layout* L, const mpcqp_vehicle* veh, int64_t B, const double* dsol,
                            const double* dAd, const double* dBd, const double* dgd, double* dxt, double* dpred,
                            double* dpdu, void* stream) {
    if (!L || !veh || !dsol || !dAd || !dBd || !dgd || !dxt || !dpred || !dpdu || B < 0)
        return set_error(MPCQP_EINVAL, "incr_shift: bad arguments");
    if (L->nx != 6 || L->nu != 2)
        return set_error(MPCQP_EUNSUPPORTED, "incr_shift: the plant model is the 6-state dynamic bicycle (nx 6, nu 2)");
    if (B == 0) return 0;
    if (int e = ensure_device(*const_cast<mpcqp_incr_layout*>(L))) return e;
    MHIPCHK(hipSetDevice(L->dev));
    const VehicleK vk = vehicle_constants(*veh);
    hipLaunchKernelGGL(k_incr_shift, dim3(grid_of(B, 128)), dim3(128), 0, (hipStream_t)stream, vk, incr_k(*L),
                       (long)B, dsol, dAd, dBd, dgd, dxt, dpred, dpdu);
    MHIPCHK(hipGetLastError());
    return 0;
}

int mpcqp_incr_warm_shift_device(int64_t B, int32_t N, int32_t nxa, int32_t nu, const double* dx, const double* dy,
                                 double* dxs, double* dys, int32_t device, void* stream) {
    if (!dx || !dxs || B < 0 || N < 1 || nxa < 1 || nu < 1 || (!dy) != (!dys) || dx == dxs || (dy && dy == dys))
        return set_error(MPCQP_EINVAL, "incr_warm_shift: bad arguments");
    if (B == 0) return 0;
    MHIPCHK(hipSetDevice(device));
    const int n = (N + 1) * nxa + N * nu, m = 2 * (N + 1) * nxa + N * nu;
    const long tx = B * (long)n;
    hipLaunchKernelGGL(k_stage_shift, dim3(grid_of(tx, 256)), dim3(256), 0, (hipStream_t)stream, tx, n, N, nxa, nu, 1,
                       dx, dxs);
    if (dy) {
        const long ty = B * (long)m;
        hipLaunchKernelGGL(k_stage_shift, dim3(grid_of(ty, 256)), dim3(256), 0, (hipStream_t)stream, ty, m, N, nxa,
                           nu, 2, dy, dys);
    }
    MHIPCHK(hipGetLastError());
    return 0;
}

int mpcqp_affine_create(int32_t nseg, const int32_t* seglen, int32_t nregimes, int32_t T, const double* base,
                        const int32_t* idx, const double* coef, int32_t device, mpcqp_affine** out) {
    if (!out || !seglen || !base || (T > 0 && (!idx || !coef)) || nseg < 1 || nseg > 3 || nregimes < 1 || T < 0)
        return set_error(MPCQP_EINVAL, "affine_create: bad arguments");
    *out = nullptr;
    auto a = std::make_unique<mpcqp_affine>();
    int L = 0, st[3] = {0, 0, 0};
    for (int s = 0; s < nseg; ++s) {
        if (seglen[s] < 0) return set_error(MPCQP_EINVAL, "affine_create: negative segment length");
        L += seglen[s];
        st[s] = L;
    }
    if (L == 0) return set_error(MPCQP_EINVAL, "affine_create: empty map");
    a->dev = device; a->L = L; a->R = nregimes; a->T = T;
    a->seg0 = st[0]; a->seg1 = nseg > 1 ? st[1] : L;
    if (nseg == 1) a->seg0 = a->seg1 = L;
    std::vector<double> vb(base, base + (size_t)nregimes * L), vc;
    std::vector<int> vi;
    if (T > 0) {
        vc.assign(coef, coef + (size_t)L * T);
        vi.assign(idx, idx + (size_t)L * T);
    } else {
        vc.assign(1, 0.0);
        vi.assign(1, -1);
    }
    for (int k : vi) a->nparam = std::max(a->nparam, k + 1);
    MHIPCHK(hipSetDevice(device));
    if (int e = upload(vb, &a->d_base)) return e;
    if (int e = upload(vc, &a->d_coef)) return e;
    if (int e = upload(vi, &a->d_idx)) return e;
    *out = a.release();
    return 0;
}

int mpcqp_affine_apply_device(const mpcqp_affine* a, int64_t B, const double* dtheta, int32_t theta_stride,
                              const int32_t* dregime, double* dout0, double* dout1, double* dout2, void* stream) {
    if (!a || B < 0 || (a->nparam > 0 && (!dtheta || theta_stride < a->nparam)) || !dout0 ||
        (a->seg1 > a->seg0 && !dout1) || (a->L > a->seg1 && !dout2))
        return set_error(MPCQP_EINVAL, "affine_apply: bad arguments (theta_stride must cover the %d parameters)",
                         a ? a->nparam : 0);
    if (B == 0) return 0;
    MHIPCHK(hipSetDevice(a->dev));
    AffineK k;
    k.L = a->L; k.R = a->R; k.T = a->T; k.seg0 = a->seg0; k.seg1 = a->seg1;
    k.base = a->d_base; k.coef = a->d_coef; k.idx = a->d_idx;
    if (a->T == 0) k.T = 0;
    hipLaunchKernelGGL(k_affine, dim3(grid_of((long)B * a->L, 256)), dim3(256), 0, (hipStream_t)stream, k, (long)B,
                       dtheta, (int)theta_stride, dregime, dout0, dout1, dout2);
    MHIPCHK(hipGetLastError());
    return 0;
}

void mpcqp_affine_free(mpcqp_affine* a) {
    if (!a) return;
    (void)hipSetDevice(a->dev);
    for (void* p : {(void*)a->d_base, (void*)a->d_coef, (void*)a->d_idx})
        if (p) (void)hipFree(p);
    delete a;
}

void mpcqp_incr_layout_free(mpcqp_incr_layout* L) {
    if (!L) return;
    if (L->d_asrc) (void)hipSetDevice(L->dev);
    for (void* p : {(void*)L->d_asrc, (void*)L->d_Atpl, (void*)L->d_ltpl, (void*)L->d_utpl, (void*)L->d_Qt})
        if (p) (void)hipFree(p);
    delete L;
}

}  // extern "C"
