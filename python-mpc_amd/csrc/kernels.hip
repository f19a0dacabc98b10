// kernels.hip -- MI355X (gfx950) device code of the batched OSQP-algorithm solver.
//
// One 256-thread workgroup per QP instance.  Per-instance data and the ADMM
// state live in LDS for the whole solve; the block-tridiagonal factor of the
// reduced KKT matrix  K = P + sigma I + A' diag(rho) A  (plan.h) is held per
// instance in a device workspace and refreshed in-kernel on every rho change.
//
// The arithmetic restates OSQP 0.6 (the reference's solver, called at
// vehicle_lateral_mpc_slack_increment.py:121,248 and Control/MPC/*.py; see
// oracle/osqp_oracle.c for the CPU restatement the tests compare with):
//   k_setup  : osqp_setup -> scale_data (Ruiz, 10 passes + cost scaling),
//              set_rho_vec (loose / equality / inequality classes)
//   k_update : osqp_update_lin_cost / osqp_update_bounds (+ update_rho_vec)
//   k_warm   : osqp_warm_start
//   k_solve  : osqp_solve -> ADMM (update_xz_tilde, update_x, update_z,
//              update_y), update_info / check_termination every
//              check_termination iterations, adapt_rho + refactorisation,
//              store_solution (unscaling)
// The only algorithmic difference from OSQP is the linear-system method:
// OSQP factors the quasi-definite KKT [[P+sI, A'], [A, -1/rho]] with QDLDL;
// here the equivalent reduced SPD system is solved by block-tridiagonal
// elimination (identical in exact arithmetic: x~ = K^{-1}(s x - q + A'(rho z - y)),
// z~ = A x~).
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace mpcqp {

#define OSQP_INFTY 1e30
#define MIN_SCALING 1e-4
#define MAX_SCALING 1e4
#define RHO_MIN 1e-6
#define RHO_MAX 1e6
#define RHO_TOL 1e-4
#define RHO_EQ_OVER_RHO_INEQ 1e3
#define DIVISION_TOL (1.0 / OSQP_INFTY)

constexpr int T = kThreads;
constexpr int S = kS;
constexpr int SS = kS * kS;

__device__ __forceinline__ double cmax(double a, double b) { return a > b ? a : b; }
__device__ __forceinline__ double cmin(double a, double b) { return a < b ? a : b; }
__device__ __forceinline__ double limit_scaling(double d) {
    d = d < MIN_SCALING ? 1.0 : d;
    return d > MAX_SCALING ? MAX_SCALING : d;
}

__device__ __forceinline__ double reduce8(double v) {
    v += __shfl_xor(v, 1);
    v += __shfl_xor(v, 2);
    v += __shfl_xor(v, 4);
    return v;
}

// block-wide max of K values (OSQP c_max semantics: NaN never wins)
template <int K>
__device__ __forceinline__ void block_max(double (&v)[K], double* red) {
#pragma unroll
    for (int k = 0; k < K; ++k)
        for (int o = 32; o > 0; o >>= 1) v[k] = cmax(v[k], __shfl_xor(v[k], o));
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < K; ++k) red[wid * K + k] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k)
        v[k] = cmax(cmax(red[k], red[K + k]), cmax(red[2 * K + k], red[3 * K + k]));
    __syncthreads();
}

template <int K>
__device__ __forceinline__ void block_sum(double (&v)[K], double* red) {
#pragma unroll
    for (int k = 0; k < K; ++k)
        for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < K; ++k) red[wid * K + k] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = (red[k] + red[K + k]) + (red[2 * K + k] + red[3 * K + k]);
    __syncthreads();
}

__device__ __forceinline__ bool block_any(bool f, int* flag) {
    if (threadIdx.x == 0) *flag = 0;
    __syncthreads();
    if (f) *flag = 1;
    __syncthreads();
    bool r = *flag != 0;
    __syncthreads();
    return r;
}

// ------------------------------------------------------------------ setup --
// osqp_setup: copy, Ruiz-scale (scale_data), classify rows (set_rho_vec).
__global__ __launch_bounds__(T) void k_setup(KParams p, const double* __restrict__ Px_in,
                                             const double* __restrict__ Ax_in,
                                             const double* __restrict__ q_in,
                                             const double* __restrict__ l_in,
                                             const double* __restrict__ u_in) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    const int tid = threadIdx.x;
    const long b = blockIdx.x;
    const int n = p.n, m = p.m, npad = p.npad, nnzP = p.nnzP, nnzA = p.nnzA;
    double* Pv = sm;
    double* Av = Pv + nnzP;
    double* qv = Av + nnzA;
    double* Dv = qv + npad;
    double* Dt = Dv + npad;
    double* Ev = Dt + npad;
    double* Et = Ev + m;
    double* red = Et + m;
    int* flag = (int*)(red + 64);

    for (int i = tid; i < nnzP; i += T) Pv[i] = Px_in[b * nnzP + i];
    for (int i = tid; i < nnzA; i += T) Av[i] = Ax_in[b * nnzA + i];
    for (int pc = tid; pc < npad; pc += T) {
        int j = p.pad_var[pc];
        qv[pc] = j >= 0 ? q_in[b * n + j] : 0.0;
        Dv[pc] = 1.0;
    }
    for (int i = tid; i < m; i += T) Ev[i] = 1.0;
    double c = 1.0;
    __syncthreads();

    for (int it = 0; it < p.scaling; ++it) {
        // compute_inf_norm_cols_KKT + limit_scaling + sqrt + reciprocal
        for (int pc = tid; pc < npad; pc += T) {
            double d = 1.0;
            if (p.pad_var[pc] >= 0) {
                double d1 = 0.0, d2 = 0.0;
                for (int e = p.psym_ptr[pc]; e < p.psym_ptr[pc + 1]; ++e) d1 = cmax(fabs(Pv[p.psym_v[e]]), d1);
                for (int e = p.acsc_ptr[pc]; e < p.acsc_ptr[pc + 1]; ++e) d2 = cmax(fabs(Av[p.acsc_v[e]]), d2);
                d = 1.0 / sqrt(limit_scaling(cmax(d1, d2)));
            }
            Dt[pc] = d;
        }
        for (int i = tid; i < m; i += T) {
            double e = 0.0;
            for (int q = p.acsr_ptr[i]; q < p.acsr_ptr[i + 1]; ++q) e = cmax(fabs(Av[p.acsr_v[q]]), e);
            Et[i] = 1.0 / sqrt(limit_scaling(e));
        }
        __syncthreads();
        // P <- D P D ; A <- E A D ; q <- D q ; D <- D Dt ; E <- E Et
        for (int v = tid; v < nnzP; v += T) {
            double x = Pv[v] * Dt[p.p_r[v]];
            Pv[v] = x * Dt[p.p_c[v]];
        }
        for (int v = tid; v < nnzA; v += T) {
            double x = Av[v] * Et[p.a_r[v]];
            Av[v] = x * Dt[p.a_c[v]];
        }
        for (int pc = tid; pc < npad; pc += T) { qv[pc] *= Dt[pc]; Dv[pc] *= Dt[pc]; }
        for (int i = tid; i < m; i += T) Ev[i] *= Et[i];
        __syncthreads();
        // cost normalisation: mean column inf-norm of P vs ||q||_inf
        double acc[1] = {0.0}, mq[1] = {0.0};
        for (int pc = tid; pc < npad; pc += T) {
            if (p.pad_var[pc] < 0) continue;
            double d1 = 0.0;
            for (int e = p.psym_ptr[pc]; e < p.psym_ptr[pc + 1]; ++e) d1 = cmax(fabs(Pv[p.psym_v[e]]), d1);
            acc[0] += d1;
            mq[0] = cmax(mq[0], fabs(qv[pc]));
        }
        block_sum(acc, red);
        block_max(mq, red);
        double ct = acc[0] / (double)n;
        double nq = limit_scaling(mq[0]);
        ct = limit_scaling(cmax(ct, nq));
        ct = 1.0 / ct;
        for (int v = tid; v < nnzP; v += T) Pv[v] *= ct;
        for (int pc = tid; pc < npad; pc += T) qv[pc] *= ct;
        c *= ct;
        __syncthreads();
    }

    // bounds: clip to +-OSQP_INFTY (python wrapper), validate, scale, classify
    bool bad = false;
    const double rho = cmin(cmax(p.rho0, RHO_MIN), RHO_MAX);
    for (int i = tid; i < m; i += T) {
        double li = cmax(l_in[b * m + i], -OSQP_INFTY);
        double ui = cmin(u_in[b * m + i], OSQP_INFTY);
        if (li > ui || li != li || ui != ui) bad = true;
        li = Ev[i] * li;
        ui = Ev[i] * ui;
        signed char t;
        if (li < -OSQP_INFTY * MIN_SCALING && ui > OSQP_INFTY * MIN_SCALING) t = -1;
        else if (ui - li < RHO_TOL) t = 1;
        else t = 0;
        p.l[b * m + i] = li;
        p.u[b * m + i] = ui;
        p.E[b * m + i] = Ev[i];
        p.ct[b * m + i] = t;
        p.z[b * m + i] = 0.0;
        p.y[b * m + i] = 0.0;
    }
    bad = block_any(bad, flag);
    for (int i = tid; i < nnzP; i += T) p.Px[b * nnzP + i] = Pv[i];
    for (int i = tid; i < nnzA; i += T) p.Ax[b * nnzA + i] = Av[i];
    for (int pc = tid; pc < npad; pc += T) {
        p.q[b * npad + pc] = qv[pc];
        p.D[b * npad + pc] = Dv[pc];
        p.x[b * npad + pc] = 0.0;
    }
    if (tid == 0) {
        p.scal[b * 4 + 0] = c;
        p.scal[b * 4 + 1] = 1.0 / c;
        p.scal[b * 4 + 2] = rho;
        p.status[b] = MPCQP_UNSOLVED_;
        p.err[b] = bad ? 1 : 0;
        p.iter[b] = 0;
        p.rho_upd[b] = 0;
    }
}

// ----------------------------------------------------------------- update --
__global__ __launch_bounds__(T) void k_update(KParams p, const double* __restrict__ q_in,
                                              const double* __restrict__ l_in,
                                              const double* __restrict__ u_in) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    int* flag = (int*)sm;
    const int tid = threadIdx.x;
    const long b = blockIdx.x;
    const int n = p.n, m = p.m, npad = p.npad;
    const double c = p.scal[b * 4 + 0];
    if (q_in)
        for (int pc = tid; pc < npad; pc += T) {
            int j = p.pad_var[pc];
            if (j >= 0) p.q[b * npad + pc] = (p.D[b * npad + pc] * q_in[b * n + j]) * c;
        }
    bool bad = false;
    if (l_in || u_in) {
        for (int i = tid; i < m; i += T) {
            const double E = p.E[b * m + i];
            double li, ui;
            if (l_in) li = cmax(l_in[b * m + i], -OSQP_INFTY);
            if (u_in) ui = cmin(u_in[b * m + i], OSQP_INFTY);
            // validation on the unscaled values when both are given (osqp_update_bounds),
            // on the scaled values otherwise (osqp_update_lower/upper_bound)
            if (l_in && u_in) {
                if (li > ui || li != li || ui != ui) bad = true;
                li = E * li;
                ui = E * ui;
            } else if (l_in) {
                li = E * li;
                ui = p.u[b * m + i];
                if (li > ui || li != li) bad = true;
            } else {
                ui = E * ui;
                li = p.l[b * m + i];
                if (li > ui || ui != ui) bad = true;
            }
            p.l[b * m + i] = li;
            p.u[b * m + i] = ui;
            signed char t;
            if (li < -OSQP_INFTY * MIN_SCALING && ui > OSQP_INFTY * MIN_SCALING) t = -1;
            else if (ui - li < RHO_TOL) t = 1;
            else t = 0;
            p.ct[b * m + i] = t;
        }
    }
    bad = block_any(bad, flag);
    if (tid == 0) {
        p.status[b] = MPCQP_UNSOLVED_;
        if (l_in || u_in) p.err[b] = bad ? 1 : 0;
    }
}

// ------------------------------------------------------------ warm start --
__global__ __launch_bounds__(T) void k_warm(KParams p, const double* __restrict__ x_in,
                                            const double* __restrict__ y_in) {
    const int tid = threadIdx.x;
    const long b = blockIdx.x;
    const int n = p.n, m = p.m, npad = p.npad;
    const double c = p.scal[b * 4 + 0];
    if (x_in)
        for (int pc = tid; pc < npad; pc += T) {
            int j = p.pad_var[pc];
            p.x[b * npad + pc] = j >= 0 ? (1.0 / p.D[b * npad + pc]) * x_in[b * n + j] : 0.0;
        }
    if (y_in)
        for (int i = tid; i < m; i += T) p.y[b * m + i] = ((1.0 / p.E[b * m + i]) * y_in[b * m + i]) * c;
    __syncthreads();
    // z = A x (scaled)
    const double* Ax = p.Ax + b * p.nnzA;
    const double* x = p.x + b * npad;
    for (int i = tid; i < m; i += T) {
        double s = 0.0;
        for (int e = p.acsr_ptr[i]; e < p.acsr_ptr[i + 1]; ++e) s += Ax[p.acsr_v[e]] * x[p.acsr_col[e]];
        p.z[b * m + i] = s;
    }
}

// ------------------------------------------------------------------ solve --
struct Lds {
    double *Av, *Pv, *xA, *xB, *qv, *rb, *xt, *zA, *zB, *yv, *lo, *up, *rv, *wv, *dyv;
    double *SP, *EK, *DK, *FK, *red;
    int* flag;
};

// Assemble K's blocks for the current rho and factor them (block LDL'):
//   S_0 = D_0,  F_k = E_k S_{k-1}^{-1},  S_k = D_k - F_k E_k',  H_{k-1} = F_k'
// storing F_k, H_k and S_k^{-1} (Gauss-Jordan, SPD, no pivoting needed).
// Returns false when a pivot is not positive (P + sigma I not PD on the
// constraint null space: OSQP reports "problem non convex").
__device__ bool factorize(const KParams& p, Lds& L, double* __restrict__ Fg, double* __restrict__ Hg,
                          double* __restrict__ Sg) {
    const int tid = threadIdx.x, i = tid >> 3, jg = tid & 7;
    const int nb = p.nb;
    bool ok = true;
    double* SP = L.SP;
    double* DK = L.DK;
    for (int k = 0; k < nb; ++k) {
        for (int e = tid; e < SS; e += T) { DK[e] = 0.0; L.EK[e] = 0.0; }
        __syncthreads();
        if (tid < S) DK[tid * S + tid] = p.pad_var[k * S + tid] >= 0 ? p.sigma : 1.0;
        __syncthreads();
        for (int t = p.asm_blk_ptr[k] + tid; t < p.asm_blk_ptr[k + 1]; t += T) {
            double acc = 0.0;
            for (int u = p.asm_term_ptr[t]; u < p.asm_term_ptr[t + 1]; ++u) {
                int r = p.term_r[u];
                if (r < 0) acc += L.Pv[p.term_a[u]];
                else acc += L.rv[r] * L.Av[p.term_a[u]] * L.Av[p.term_b[u]];
            }
            int tg = p.asm_tgt[t];
            if (tg < SS) DK[tg] += acc;
            else L.EK[tg - SS] += acc;
        }
        __syncthreads();
        if (k > 0) {
            // F = E S_prev^{-1}
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) {
                const int j = jg + 8 * cc;
                double s = 0.0;
                for (int l = 0; l < S; ++l) s += L.EK[i * S + l] * SP[l * S + j];
                L.FK[i * S + j] = s;
            }
            __syncthreads();
            // S = D - F E'
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) {
                const int j = jg + 8 * cc;
                double s = 0.0;
                for (int l = 0; l < S; ++l) s += L.FK[i * S + l] * L.EK[j * S + l];
                DK[i * S + j] -= s;
                Fg[(long)k * SS + i * S + j] = L.FK[i * S + j];
                Hg[(long)(k - 1) * SS + j * S + i] = L.FK[i * S + j];
            }
            __syncthreads();
        }
        // in-place Gauss-Jordan inverse of the SPD tile
        for (int pv = 0; pv < S; ++pv) {
            const double piv = DK[pv * S + pv];
            const double colv = DK[i * S + pv];
            double rowv[4];
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) rowv[cc] = DK[pv * S + jg + 8 * cc];
            __syncthreads();
            if (!(piv > 0.0)) ok = false;
            const double d = 1.0 / piv;
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) {
                const int j = jg + 8 * cc;
                double v;
                if (i == pv) v = (j == pv) ? d : rowv[cc] * d;
                else if (j == pv) v = -colv * d;
                else v = DK[i * S + j] - colv * (rowv[cc] * d);
                DK[i * S + j] = v;
            }
            __syncthreads();
        }
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
            const int j = jg + 8 * cc;
            Sg[(long)k * SS + i * S + j] = DK[i * S + j];
        }
        double* t = SP; SP = DK; DK = t;
        __syncthreads();
    }
    L.SP = SP; L.DK = DK;
    return ok;
}

// xt = K^{-1} rb  (rb is overwritten by the forward sweep)
__device__ __forceinline__ void bt_solve(const KParams& p, double* __restrict__ rb, double* __restrict__ xt,
                                         const double* __restrict__ Fg, const double* __restrict__ Hg,
                                         const double* __restrict__ Sg) {
    const int tid = threadIdx.x, i = tid >> 3, jg = tid & 7;
    const int nb = p.nb;
    for (int k = 1; k < nb; ++k) {
        const double* F = Fg + (long)k * SS + i * S;
        const double* v = rb + (k - 1) * S;
        double s = F[jg] * v[jg] + F[jg + 8] * v[jg + 8] + F[jg + 16] * v[jg + 16] + F[jg + 24] * v[jg + 24];
        s = reduce8(s);
        if (jg == 0) rb[k * S + i] -= s;
        __syncthreads();
    }
    for (int k = 0; k < nb; ++k) {
        const double* Si = Sg + (long)k * SS + i * S;
        const double* v = rb + k * S;
        double s = Si[jg] * v[jg] + Si[jg + 8] * v[jg + 8] + Si[jg + 16] * v[jg + 16] + Si[jg + 24] * v[jg + 24];
        s = reduce8(s);
        if (jg == 0) xt[k * S + i] = s;
    }
    __syncthreads();
    for (int k = nb - 2; k >= 0; --k) {
        const double* H = Hg + (long)k * SS + i * S;
        const double* v = xt + (k + 1) * S;
        double s = H[jg] * v[jg] + H[jg + 8] * v[jg + 8] + H[jg + 16] * v[jg + 16] + H[jg + 24] * v[jg + 24];
        s = reduce8(s);
        if (jg == 0) xt[k * S + i] -= s;
        __syncthreads();
    }
}

struct Res {  // update_info results (scaled-space and unscaled norms)
    double pri, dua, nz, nax, nq, naty, npx;               // termination (unscaled by E/D/c)
    double rpri, rdua, rz, rax, rq, raty, rpx;             // rho estimate (scaled space)
};

__device__ void update_info(const KParams& p, Lds& L, const double* x, const double* z, long b, double cinv,
                            Res& R) {
    const int tid = threadIdx.x, m = p.m, npad = p.npad;
    const double* Eg = p.E + b * m;
    const double* Dg = p.D + b * npad;
    double v[14];
#pragma unroll
    for (int k = 0; k < 14; ++k) v[k] = 0.0;
    for (int i = tid; i < m; i += T) {
        double ax = 0.0;
        for (int e = p.acsr_ptr[i]; e < p.acsr_ptr[i + 1]; ++e) ax += L.Av[p.acsr_v[e]] * x[p.acsr_col[e]];
        const double pr = ax - z[i];
        const double ei = 1.0 / Eg[i];
        v[0] = cmax(v[0], fabs(ei * pr));
        v[2] = cmax(v[2], fabs(ei * z[i]));
        v[3] = cmax(v[3], fabs(ei * ax));
        v[7] = cmax(v[7], fabs(pr));
        v[9] = cmax(v[9], fabs(z[i]));
        v[10] = cmax(v[10], fabs(ax));
    }
    for (int pc = tid; pc < npad; pc += T) {
        if (p.pad_var[pc] < 0) continue;
        double px = 0.0, aty = 0.0;
        for (int e = p.psym_ptr[pc]; e < p.psym_ptr[pc + 1]; ++e) px += L.Pv[p.psym_v[e]] * x[p.psym_col[e]];
        for (int e = p.acsc_ptr[pc]; e < p.acsc_ptr[pc + 1]; ++e) aty += L.Av[p.acsc_v[e]] * L.yv[p.acsc_row[e]];
        const double d = (L.qv[pc] + px) + aty;
        const double di = 1.0 / Dg[pc];
        v[1] = cmax(v[1], fabs(di * d));
        v[4] = cmax(v[4], fabs(di * L.qv[pc]));
        v[5] = cmax(v[5], fabs(di * aty));
        v[6] = cmax(v[6], fabs(di * px));
        v[8] = cmax(v[8], fabs(d));
        v[11] = cmax(v[11], fabs(L.qv[pc]));
        v[12] = cmax(v[12], fabs(aty));
        v[13] = cmax(v[13], fabs(px));
    }
    block_max(v, L.red);
    if (p.scaling && !p.scaled_term) {
        R.pri = v[0]; R.dua = cinv * v[1];
        R.nz = v[2]; R.nax = v[3]; R.nq = v[4]; R.naty = v[5]; R.npx = v[6];
    } else {
        R.pri = v[7]; R.dua = v[8];
        R.nz = v[9]; R.nax = v[10]; R.nq = v[11]; R.naty = v[12]; R.npx = v[13];
    }
    R.rpri = v[7]; R.rdua = v[8]; R.rz = v[9]; R.rax = v[10]; R.rq = v[11]; R.raty = v[12]; R.rpx = v[13];
    if (p.m == 0) R.pri = 0.0;
}

__device__ bool is_primal_infeasible(const KParams& p, Lds& L, long b, double eps) {
    const int tid = threadIdx.x, m = p.m, npad = p.npad;
    const bool unscale = p.scaling && !p.scaled_term;
    const double* Eg = p.E + b * m;
    double nd[1] = {0.0};
    for (int i = tid; i < m; i += T) {
        double d = L.dyv[i];
        if (L.up[i] > OSQP_INFTY * MIN_SCALING) {
            d = (L.lo[i] < -OSQP_INFTY * MIN_SCALING) ? 0.0 : cmin(d, 0.0);
        } else if (L.lo[i] < -OSQP_INFTY * MIN_SCALING) {
            d = cmax(d, 0.0);
        }
        L.dyv[i] = d;
        nd[0] = cmax(nd[0], fabs(unscale ? Eg[i] * d : d));
    }
    block_max(nd, L.red);  // contains a barrier: dyv is consistent afterwards
    const double norm_dy = nd[0];
    if (!(norm_dy > eps)) return false;
    double s[1] = {0.0};
    for (int i = tid; i < m; i += T) s[0] += L.up[i] * cmax(L.dyv[i], 0.0) + L.lo[i] * cmin(L.dyv[i], 0.0);
    block_sum(s, L.red);
    if (!(s[0] < eps * norm_dy)) return false;
    const double* Dg = p.D + b * npad;
    double na[1] = {0.0};
    for (int pc = tid; pc < npad; pc += T) {
        if (p.pad_var[pc] < 0) continue;
        double a = 0.0;
        for (int e = p.acsc_ptr[pc]; e < p.acsc_ptr[pc + 1]; ++e) a += L.Av[p.acsc_v[e]] * L.dyv[p.acsc_row[e]];
        if (unscale) a *= 1.0 / Dg[pc];
        na[0] = cmax(na[0], fabs(a));
    }
    block_max(na, L.red);
    return na[0] < eps * norm_dy;
}

// dx lives in L.rb (x - x_prev of the last iteration)
__device__ bool is_dual_infeasible(const KParams& p, Lds& L, const double* x, long b, double c, double eps) {
    const int tid = threadIdx.x, m = p.m, npad = p.npad;
    const bool unscale = p.scaling && !p.scaled_term;
    const double* Dg = p.D + b * npad;
    const double* Eg = p.E + b * m;
    const double cs = unscale ? c : 1.0;
    double v[2] = {0.0, 0.0};
    for (int pc = tid; pc < npad; pc += T) {
        if (p.pad_var[pc] < 0) continue;
        v[0] = cmax(v[0], fabs(unscale ? Dg[pc] * L.rb[pc] : L.rb[pc]));
    }
    block_max(v, L.red);
    const double norm_dx = v[0];
    if (!(norm_dx > eps)) return false;
    double s[1] = {0.0};
    for (int pc = tid; pc < npad; pc += T)
        if (p.pad_var[pc] >= 0) s[0] += L.qv[pc] * L.rb[pc];
    block_sum(s, L.red);
    if (!(s[0] < cs * eps * norm_dx)) return false;
    double np[1] = {0.0};
    for (int pc = tid; pc < npad; pc += T) {
        if (p.pad_var[pc] < 0) continue;
        double a = 0.0;
        for (int e = p.psym_ptr[pc]; e < p.psym_ptr[pc + 1]; ++e) a += L.Pv[p.psym_v[e]] * L.rb[p.psym_col[e]];
        if (unscale) a *= 1.0 / Dg[pc];
        np[0] = cmax(np[0], fabs(a));
    }
    block_max(np, L.red);
    if (!(np[0] < cs * eps * norm_dx)) return false;
    bool viol = false;
    for (int i = tid; i < m; i += T) {
        double a = 0.0;
        for (int e = p.acsr_ptr[i]; e < p.acsr_ptr[i + 1]; ++e) a += L.Av[p.acsr_v[e]] * L.rb[p.acsr_col[e]];
        if (unscale) a *= 1.0 / Eg[i];
        if ((L.up[i] < OSQP_INFTY * MIN_SCALING && a > eps * norm_dx) ||
            (L.lo[i] > -OSQP_INFTY * MIN_SCALING && a < -eps * norm_dx))
            viol = true;
    }
    return !block_any(viol, L.flag);
}

// returns 1 when the solver terminates; sets *status
__device__ int check_termination(const KParams& p, Lds& L, const double* x, long b, double c, double cinv,
                                 const Res& R, bool approximate, int* status, double* obj) {
    double eps_abs = p.eps_abs, eps_rel = p.eps_rel, eps_pinf = p.eps_pinf, eps_dinf = p.eps_dinf;
    if (R.pri > OSQP_INFTY || R.dua > OSQP_INFTY) {
        *status = MPCQP_NON_CVX_;
        *obj = __builtin_nan("");
        return 1;
    }
    if (approximate) { eps_abs *= 10; eps_rel *= 10; eps_pinf *= 10; eps_dinf *= 10; }
    bool prim_ok = false, dual_ok = false, prim_inf = false, dual_inf = false;
    const bool unscale = p.scaling && !p.scaled_term;
    if (p.m == 0) prim_ok = true;
    else {
        const double ep = eps_abs + eps_rel * cmax(R.nz, R.nax);
        if (R.pri < ep) prim_ok = true;
        else prim_inf = is_primal_infeasible(p, L, b, eps_pinf);
    }
    double mx = cmax(cmax(R.nq, R.naty), R.npx);
    if (unscale) mx *= cinv;
    const double ed = eps_abs + eps_rel * mx;
    if (R.dua < ed) dual_ok = true;
    else dual_inf = is_dual_infeasible(p, L, x, b, c, eps_dinf);
    if (prim_ok && dual_ok) {
        *status = approximate ? MPCQP_SOLVED_INACCURATE_ : MPCQP_SOLVED_;
        return 1;
    }
    if (prim_inf) {
        *status = approximate ? MPCQP_PRIMAL_INFEASIBLE_INACCURATE_ : MPCQP_PRIMAL_INFEASIBLE_;
        if (unscale)
            for (int i = threadIdx.x; i < p.m; i += T) L.dyv[i] *= p.E[b * p.m + i];
        __syncthreads();
        *obj = OSQP_INFTY;
        return 1;
    }
    if (dual_inf) {
        *status = approximate ? MPCQP_DUAL_INFEASIBLE_INACCURATE_ : MPCQP_DUAL_INFEASIBLE_;
        if (unscale)
            for (int pc = threadIdx.x; pc < p.npad; pc += T) L.rb[pc] *= p.D[b * p.npad + pc];
        __syncthreads();
        *obj = -OSQP_INFTY;
        return 1;
    }
    return 0;
}

__device__ __forceinline__ void set_rho_vec(const KParams& p, Lds& L, const signed char* ct, double rho) {
    for (int i = threadIdx.x; i < p.m; i += T) {
        const signed char t = ct[i];
        L.rv[i] = t < 0 ? RHO_MIN : (t > 0 ? RHO_EQ_OVER_RHO_INEQ * rho : rho);
    }
}

__global__ __launch_bounds__(T) void k_solve(KParams p, double* __restrict__ xo, double* __restrict__ yo,
                                             int factor_only) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    const int tid = threadIdx.x;
    const long b = blockIdx.x;
    const int n = p.n, m = p.m, npad = p.npad, nnzP = p.nnzP, nnzA = p.nnzA;
    Lds L;
    L.Av = sm;
    L.Pv = L.Av + nnzA;
    L.xA = L.Pv + nnzP;
    L.xB = L.xA + npad;
    L.qv = L.xB + npad;
    L.rb = L.qv + npad;
    L.xt = L.rb + npad;
    L.zA = L.xt + npad;
    L.zB = L.zA + m;
    L.yv = L.zB + m;
    L.lo = L.yv + m;
    L.up = L.lo + m;
    L.rv = L.up + m;
    L.wv = L.rv + m;
    L.dyv = L.wv + m;
    L.SP = L.dyv + m;
    L.EK = L.SP + SS;
    L.DK = L.EK + SS;
    L.FK = L.DK + SS;
    L.red = L.FK + SS;
    L.flag = (int*)(L.red + 128);

    double* Fg = p.F + b * (long)p.nb * SS;
    double* Hg = p.H + b * (long)p.nb * SS;
    double* Sg = p.Si + b * (long)p.nb * SS;
    const signed char* ctg = p.ct + b * m;

    if (p.err[b]) {  // invalid data: leave NaN outputs, status unchanged semantics
        for (int j = tid; j < n; j += T) if (xo) xo[b * n + j] = __builtin_nan("");
        for (int i = tid; i < m; i += T) if (yo) yo[b * m + i] = __builtin_nan("");
        if (tid == 0) p.status[b] = MPCQP_NON_CVX_;
        return;
    }

    const double c = p.scal[b * 4 + 0], cinv = p.scal[b * 4 + 1];
    double rho = p.scal[b * 4 + 2];
    for (int i = tid; i < nnzA; i += T) L.Av[i] = p.Ax[b * nnzA + i];
    for (int i = tid; i < nnzP; i += T) L.Pv[i] = p.Px[b * nnzP + i];
    const bool warm = p.warm_start != 0;
    for (int pc = tid; pc < npad; pc += T) {
        L.qv[pc] = p.q[b * npad + pc];
        L.xA[pc] = warm ? p.x[b * npad + pc] : 0.0;
        L.xB[pc] = 0.0;
        L.rb[pc] = 0.0;
        L.xt[pc] = 0.0;
    }
    for (int i = tid; i < m; i += T) {
        L.zA[i] = warm ? p.z[b * m + i] : 0.0;
        L.zB[i] = 0.0;
        L.yv[i] = warm ? p.y[b * m + i] : 0.0;
        L.lo[i] = p.l[b * m + i];
        L.up[i] = p.u[b * m + i];
        L.dyv[i] = 0.0;
    }
    set_rho_vec(p, L, ctg, rho);
    __syncthreads();

    if (!factorize(p, L, Fg, Hg, Sg)) {
        for (int j = tid; j < n; j += T) if (xo) xo[b * n + j] = __builtin_nan("");
        for (int i = tid; i < m; i += T) if (yo) yo[b * m + i] = __builtin_nan("");
        if (tid == 0) p.status[b] = MPCQP_NON_CVX_;
        return;
    }
    if (factor_only) return;

    const double sigma = p.sigma, alpha = p.alpha;
    double* x = L.xA;
    double* xp = L.xB;
    double* z = L.zA;
    double* zp = L.zB;
    int status = MPCQP_UNSOLVED_;
    int rho_updates = 0;
    double obj = 0.0, rho_est = rho;
    Res R{};
    bool can_check = false;
    int iter;
    int info_iter = 0;
    for (iter = 1; iter <= p.max_iter; ++iter) {
        { double* t = x; x = xp; xp = t; }
        { double* t = z; z = zp; zp = t; }
        // w = rho z_prev - y
        for (int i = tid; i < m; i += T) L.wv[i] = L.rv[i] * zp[i] - L.yv[i];
        __syncthreads();
        // rhs = sigma x_prev - q + A' w
        for (int pc = tid; pc < npad; pc += T) {
            double r = 0.0;
            if (p.pad_var[pc] >= 0) {
                double acc = 0.0;
                for (int e = p.acsc_ptr[pc]; e < p.acsc_ptr[pc + 1]; ++e) acc += L.Av[p.acsc_v[e]] * L.wv[p.acsc_row[e]];
                r = (sigma * xp[pc] - L.qv[pc]) + acc;
            }
            L.rb[pc] = r;
        }
        __syncthreads();
        bt_solve(p, L.rb, L.xt, Fg, Hg, Sg);
        // z~ = A x~ ; update_z (relaxed + projected) ; update_y
        for (int i = tid; i < m; i += T) {
            double zt = 0.0;
            for (int e = p.acsr_ptr[i]; e < p.acsr_ptr[i + 1]; ++e) zt += L.Av[p.acsr_v[e]] * L.xt[p.acsr_col[e]];
            const double rinv = 1.0 / L.rv[i];
            const double zr = alpha * zt + (1.0 - alpha) * zp[i];
            const double zn = cmin(cmax(zr + rinv * L.yv[i], L.lo[i]), L.up[i]);
            const double dy = L.rv[i] * (zr - zn);
            z[i] = zn;
            L.dyv[i] = dy;
            L.yv[i] += dy;
        }
        // update_x ; delta_x kept in rb
        for (int pc = tid; pc < npad; pc += T) {
            const double xn = alpha * L.xt[pc] + (1.0 - alpha) * xp[pc];
            x[pc] = xn;
            L.rb[pc] = xn - xp[pc];
        }
        __syncthreads();

        can_check = p.check_term && (iter % p.check_term == 0);
        const bool do_rho = p.adaptive_rho && p.rho_interval && (iter % p.rho_interval == 0);
        if (can_check || do_rho) {
            update_info(p, L, x, z, b, cinv, R);
            info_iter = iter;
        }
        if (can_check) {
            if (check_termination(p, L, x, b, c, cinv, R, false, &status, &obj)) break;
        }
        if (do_rho) {
            double pr = R.rpri / (cmax(R.rz, R.rax) + DIVISION_TOL);
            double du = R.rdua / (cmax(cmax(R.rq, R.raty), R.rpx) + DIVISION_TOL);
            double rn = rho * sqrt(pr / (du + DIVISION_TOL));
            rn = cmin(cmax(rn, RHO_MIN), RHO_MAX);
            rho_est = rn;
            if (rn > rho * p.rho_tol || rn < rho / p.rho_tol) {
                rho = cmin(cmax(rn, RHO_MIN), RHO_MAX);
                set_rho_vec(p, L, ctg, rho);
                __syncthreads();
                rho_updates++;
                if (!factorize(p, L, Fg, Hg, Sg)) { status = MPCQP_NON_CVX_; break; }
            }
        }
    }
    if (!can_check && status == MPCQP_UNSOLVED_) {
        update_info(p, L, x, z, b, cinv, R);
        info_iter = iter - 1;
        check_termination(p, L, x, b, c, cinv, R, false, &status, &obj);
    }
    const bool has_sol = !(status == MPCQP_PRIMAL_INFEASIBLE_ || status == MPCQP_PRIMAL_INFEASIBLE_INACCURATE_ ||
                           status == MPCQP_DUAL_INFEASIBLE_ || status == MPCQP_DUAL_INFEASIBLE_INACCURATE_ ||
                           status == MPCQP_NON_CVX_);
    if (has_sol) {
        // compute_obj_val: (x'Px/2 + q'x) / c  (P upper triangle)
        double s[1] = {0.0};
        for (int v = tid; v < nnzP; v += T) {
            const int r = p.p_r[v], cc = p.p_c[v];
            s[0] += (r == cc) ? 0.5 * L.Pv[v] * x[r] * x[r] : L.Pv[v] * x[r] * x[cc];
        }
        for (int pc = tid; pc < npad; pc += T) s[0] += L.qv[pc] * x[pc];
        block_sum(s, L.red);
        obj = p.scaling ? s[0] * cinv : s[0];
    }
    if (status == MPCQP_UNSOLVED_) {
        if (!check_termination(p, L, x, b, c, cinv, R, true, &status, &obj)) status = MPCQP_MAX_ITER_REACHED_;
    }
    {
        double pr = R.rpri / (cmax(R.rz, R.rax) + DIVISION_TOL);
        double du = R.rdua / (cmax(cmax(R.rq, R.raty), R.rpx) + DIVISION_TOL);
        double rn = rho * sqrt(pr / (du + DIVISION_TOL));
        rho_est = cmin(cmax(rn, RHO_MIN), RHO_MAX);
    }
    const bool has_sol2 = !(status == MPCQP_PRIMAL_INFEASIBLE_ || status == MPCQP_PRIMAL_INFEASIBLE_INACCURATE_ ||
                            status == MPCQP_DUAL_INFEASIBLE_ || status == MPCQP_DUAL_INFEASIBLE_INACCURATE_ ||
                            status == MPCQP_NON_CVX_);
    // store_solution + certificates
    double nrm[2] = {0.0, 0.0};
    if (!has_sol2) {
        for (int i = tid; i < m; i += T) nrm[0] = cmax(nrm[0], fabs(L.dyv[i]));
        for (int pc = tid; pc < npad; pc += T) nrm[1] = cmax(nrm[1], fabs(L.rb[pc]));
        block_max(nrm, L.red);
    }
    const bool pinf = status == MPCQP_PRIMAL_INFEASIBLE_ || status == MPCQP_PRIMAL_INFEASIBLE_INACCURATE_;
    const bool dinf = status == MPCQP_DUAL_INFEASIBLE_ || status == MPCQP_DUAL_INFEASIBLE_INACCURATE_;
    for (int pc = tid; pc < npad; pc += T) {
        const int j = p.pad_var[pc];
        double xv = x[pc];
        double dx = L.rb[pc];
        if (dinf) dx *= 1.0 / nrm[1];
        if (j >= 0) {
            if (xo) xo[b * n + j] = has_sol2 ? (p.scaling ? p.D[b * npad + pc] * xv : xv) : __builtin_nan("");
            p.dxc[b * n + j] = dx;
        }
        p.x[b * npad + pc] = has_sol2 ? xv : 0.0;
    }
    for (int i = tid; i < m; i += T) {
        double yv = L.yv[i];
        double dy = L.dyv[i];
        if (pinf) dy *= 1.0 / nrm[0];
        if (yo) yo[b * m + i] = has_sol2 ? (p.scaling ? (p.E[b * m + i] * yv) * cinv : yv) : __builtin_nan("");
        p.dyc[b * m + i] = dy;
        p.y[b * m + i] = has_sol2 ? yv : 0.0;
        p.z[b * m + i] = has_sol2 ? z[i] : 0.0;
    }
    if (tid == 0) {
        p.status[b] = status;
        p.iter[b] = info_iter;
        p.rho_upd[b] = rho_updates;
        p.obj[b] = obj;
        p.pri[b] = R.pri;
        p.dua[b] = R.dua;
        p.rho_est[b] = rho_est;
        p.scal[b * 4 + 2] = rho;
    }
}

// ------------------------------------------------------------ launchers --
size_t lds_setup_bytes(const KParams& p) {
    return sizeof(double) * ((size_t)p.nnzP + p.nnzA + 3 * (size_t)p.npad + 2 * (size_t)p.m + 64) + 16;
}
size_t lds_solve_bytes(const KParams& p) {
    return sizeof(double) * ((size_t)p.nnzA + p.nnzP + 5 * (size_t)p.npad + 8 * (size_t)p.m + 4 * SS + 128) + 16;
}

hipError_t launch_setup(const KParams& p, long B, const double* Px, const double* Ax, const double* q,
                        const double* l, const double* u, hipStream_t st) {
    size_t lds = lds_setup_bytes(p);
    hipError_t e = hipFuncSetAttribute((const void*)k_setup, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_setup, dim3((unsigned)B), dim3(T), lds, st, p, Px, Ax, q, l, u);
    return hipGetLastError();
}
hipError_t launch_update(const KParams& p, long B, const double* q, const double* l, const double* u,
                         hipStream_t st) {
    hipLaunchKernelGGL(k_update, dim3((unsigned)B), dim3(T), 64, st, p, q, l, u);
    return hipGetLastError();
}
hipError_t launch_warm(const KParams& p, long B, const double* x, const double* y, hipStream_t st) {
    hipLaunchKernelGGL(k_warm, dim3((unsigned)B), dim3(T), 0, st, p, x, y);
    return hipGetLastError();
}
hipError_t launch_solve(const KParams& p, long B, double* xo, double* yo, int factor_only, hipStream_t st) {
    size_t lds = lds_solve_bytes(p);
    hipError_t e = hipFuncSetAttribute((const void*)k_solve, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_solve, dim3((unsigned)B), dim3(T), lds, st, p, xo, yo, factor_only);
    return hipGetLastError();
}

}  // namespace mpcqp
