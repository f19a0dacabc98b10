// kernels.hip -- MI355X (gfx950) data kernels of the batched OSQP-algorithm solver:
// setup (scaling), update, warm start.  The ADMM kernel is in solve.hip.
//
// One 256-thread workgroup per QP instance.
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

#include <algorithm>

#include "device_common.h"
#include "setup_r.h"
#include "setup_wide.h"
#include "wave_util.h"

namespace mpcqp {

// ------------------------------------------------------------------ setup --
// osqp_setup: copy, Ruiz-scale (scale_data), classify rows (set_rho_vec).
// The plan's index arrays from pad_var to a_c (one contiguous span of the flat plan,
// api.hip::upload_plan) are staged in LDS once, so the ten scaling passes chase
// LDS indices instead of dependent global loads.
__host__ __device__ inline long setup_span(const KParams& p) { return (long)(p.asm_blk_ptr - p.pad_var); }

// KEEP: a matrix update (k_unscale_mat): scale afresh, leave x, z, y, the row classes and rho
template <bool STAGE, bool KEEP>  // STAGE false: plans whose index span does not fit in LDS read it from the plan
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
    int* ix = STAGE ? flag + 4 : (int*)p.pad_var;  // the staged index span
    if (STAGE) {
        const long span = setup_span(p);
        for (long o = tid; o < span; o += T) ix[o] = p.pad_var[o];
    }
    auto rebase = [&](const int* a) __attribute__((always_inline)) { return ix + (a - p.pad_var); };
    const int *pad_var = ix, *psym_ptr = rebase(p.psym_ptr), *psym_v = rebase(p.psym_v);
    const int *acsc_ptr = rebase(p.acsc_ptr), *acsc_v = rebase(p.acsc_v);
    const int *acsr_ptr = rebase(p.acsr_ptr), *acsr_v = rebase(p.acsr_v);
    const int *p_r = rebase(p.p_r), *p_c = rebase(p.p_c), *a_r = rebase(p.a_r), *a_c = rebase(p.a_c);

    const long bm = p.mat_shared ? 0 : b;  // LTI batches: one P, A for every instance
    for (int i = tid; i < nnzP; i += T) Pv[i] = Px_in[bm * nnzP + i];
    for (int i = tid; i < nnzA; i += T) Av[i] = Ax_in[bm * nnzA + i];
    __syncthreads();  // the staged indices
    for (int pc = tid; pc < npad; pc += T) {
        int j = pad_var[pc];
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
            if (pad_var[pc] >= 0) {
                double d1 = 0.0, d2 = 0.0;
                for (int e = psym_ptr[pc]; e < psym_ptr[pc + 1]; ++e) d1 = cmax(fabs(Pv[psym_v[e]]), d1);
                for (int e = acsc_ptr[pc]; e < acsc_ptr[pc + 1]; ++e) d2 = cmax(fabs(Av[acsc_v[e]]), d2);
                d = 1.0 / sqrt(limit_scaling(cmax(d1, d2)));
            }
            Dt[pc] = d;
        }
        for (int i = tid; i < m; i += T) {
            double e = 0.0;
            for (int q = acsr_ptr[i]; q < acsr_ptr[i + 1]; ++q) e = cmax(fabs(Av[acsr_v[q]]), e);
            Et[i] = 1.0 / sqrt(limit_scaling(e));
        }
        __syncthreads();
        // P <- D P D ; A <- E A D ; q <- D q ; D <- D Dt ; E <- E Et
        for (int v = tid; v < nnzP; v += T) {
            double x = Pv[v] * Dt[p_r[v]];
            Pv[v] = x * Dt[p_c[v]];
        }
        for (int v = tid; v < nnzA; v += T) {
            double x = Av[v] * Et[a_r[v]];
            Av[v] = x * Dt[a_c[v]];
        }
        for (int pc = tid; pc < npad; pc += T) { qv[pc] *= Dt[pc]; Dv[pc] *= Dt[pc]; }
        for (int i = tid; i < m; i += T) Ev[i] *= Et[i];
        __syncthreads();
        // cost normalisation: mean column inf-norm of P vs ||q||_inf
        double acc[1] = {0.0}, mq[1] = {0.0};
        for (int pc = tid; pc < npad; pc += T) {
            if (pad_var[pc] < 0) continue;
            double d1 = 0.0;
            for (int e = psym_ptr[pc]; e < psym_ptr[pc + 1]; ++e) d1 = cmax(fabs(Pv[psym_v[e]]), d1);
            acc[0] += d1;
            mq[0] = cmax(mq[0], fabs(qv[pc]));
        }
        block_sum<T>(acc, red);
        block_max<T>(mq, red);
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
        if (!KEEP) {
            p.ct[b * m + i] = t;
            p.z[b * m + i] = 0.0;
            p.y[b * m + i] = 0.0;
        }
    }
    bad = block_any<T>(bad, flag);
    for (int i = tid; i < nnzP; i += T) p.Px[b * nnzP + i] = Pv[i];
    // scaled A in the padded-CSC order the solve kernels keep in LDS (one linear load there)
    for (int e = tid; e < nnzA; e += T) p.Ax[b * nnzA + e] = Av[acsc_v[e]];
    for (int pc = tid; pc < npad; pc += T) {
        p.q[b * npad + pc] = qv[pc];
        p.D[b * npad + pc] = Dv[pc];
        if (!KEEP) p.x[b * npad + pc] = 0.0;
    }
    if (tid == 0) {
        p.scal[b * 4 + 0] = c;
        p.scal[b * 4 + 1] = 1.0 / c;
        p.status[b] = MPCQP_UNSOLVED_;
        p.err[b] = bad ? 1 : 0;
        p.ffresh[b] = 0;
        if (!KEEP) {
            p.scal[b * 4 + 2] = rho;
            p.iter[b] = 0;
            p.rho_upd[b] = 0;
        }
    }
}

// ------------------------------------------------- setup, register lists --
// setup_r.h::setup_r_body with 256 threads: one padded column and one row per thread
template <int K, int KP, int AS, int PS, bool KEEP>
__global__ __launch_bounds__(T) void k_setup_r(KParams p, const double* __restrict__ Px_in,
                                               const double* __restrict__ Ax_in,
                                               const double* __restrict__ q_in,
                                               const double* __restrict__ l_in,
                                               const double* __restrict__ u_in) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    setup_r_body<T, K, KP, 1, AS, PS, KEEP>(p, (long)blockIdx.x, Px_in, Ax_in, q_in, l_in, u_in, sm);
}

// the same for the long-horizon plans (cfg 5: npad 544, m 916, nnz(A) 2666), setup_wide.h:
// 1024 threads with one padded column, one row and three A values each for a few instances
// (one instance per CU), 512 threads with two of each and six A values for batches (two
// instances per CU: the setup is latency-bound) -- the register-list setup instead of
// k_setup's index chains (one cfg-5 instance: ten Ruiz passes ~165 us there)
constexpr int TWIDE = 1024;
template <int TT, int CS, int AS, bool KEEP, bool WARM = false>
__global__ __launch_bounds__(TT, TT == 512 ? 4 : 1) void k_setup_wide(KParams p, const double* __restrict__ Px_in,
                                                                      const double* __restrict__ Ax_in,
                                                                      const double* __restrict__ q_in,
                                                                      const double* __restrict__ l_in,
                                                                      const double* __restrict__ u_in,
                                                                      const double* __restrict__ x0,
                                                                      const double* __restrict__ y0) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    setup_wide_body<TT, CS, CS, 8, 4, AS, CS, KEEP, WARM>(p, (long)blockIdx.x, Px_in, Ax_in, q_in, l_in, u_in, sm,
                                                          x0, y0);
}

// ------------------------------------------------------- matrix update --
// osqp_update_P / osqp_update_A / osqp_update_P_A (OSQP 0.6; the call the reference's
// commented-out update(Px=, Px_idx=) at vehicle_lateral_mpc_slack_increment.py:236 would
// make): unscale_data -- P <- cinv Dinv P Dinv, q <- Dinv (cinv q), A <- Einv A Dinv,
// l, u <- Einv (l, u), one rounding per factor in OSQP's order -- into the setup inputs
// (user order), then the new values at their indices (none: all nnz); launch_update_mat
// then scales them afresh with k_setup(_r)<KEEP>, which leaves x, z, y, the row classes
// and rho as OSQP 0.6 does.  Dinv / Einv as OSQP forms them (vec_ew_recipr: 1 / D).
__global__ __launch_bounds__(T) void k_unscale_mat(KParams p, double* __restrict__ Px_o, double* __restrict__ Ax_o,
                                                   double* __restrict__ q_o, double* __restrict__ l_o,
                                                   double* __restrict__ u_o, const double* __restrict__ Px_new,
                                                   const int* __restrict__ Px_idx, int nP,
                                                   const double* __restrict__ Ax_new,
                                                   const int* __restrict__ Ax_idx, int nA) {
    const int tid = threadIdx.x;
    const long b = blockIdx.x;
    const int n = p.n, m = p.m, npad = p.npad, nnzP = p.nnzP, nnzA = p.nnzA;
    const double* D = p.D + b * npad;
    const double* E = p.E + b * m;
    const bool sc = p.scaling != 0;
    const double cinv = p.scal[b * 4 + 1];
    for (int v = tid; v < nnzP; v += T) {
        double x = p.Px[b * nnzP + v];
        if (sc) {
            x *= cinv;
            x *= 1.0 / D[p.p_r[v]];
            x *= 1.0 / D[p.p_c[v]];
        }
        Px_o[b * nnzP + v] = x;
    }
    for (int e = tid; e < nnzA; e += T) {  // the workspace keeps A in padded-CSC order
        const int v = p.acsc_v[e];
        double x = p.Ax[b * nnzA + e];
        if (sc) {
            x *= 1.0 / E[p.acsc_row[e]];
            x *= 1.0 / D[p.a_c[v]];
        }
        Ax_o[b * nnzA + v] = x;
    }
    for (int pc = tid; pc < npad; pc += T) {
        const int j = p.pad_var[pc];
        if (j < 0) continue;
        double x = p.q[b * npad + pc];
        if (sc) {
            x *= cinv;
            x *= 1.0 / D[pc];
        }
        q_o[b * n + j] = x;
    }
    for (int i = tid; i < m; i += T) {
        double li = p.l[b * m + i], ui = p.u[b * m + i];
        if (sc) {
            const double ei = 1.0 / E[i];
            li *= ei;
            ui *= ei;
        }
        l_o[b * m + i] = li;
        u_o[b * m + i] = ui;
    }
    __syncthreads();
    // the new values (indices unique: the host keeps the last of repeated ones, as OSQP's
    // sequential loop does)
    if (Px_new)
        for (int k = tid; k < nP; k += T) Px_o[b * nnzP + (Px_idx ? Px_idx[k] : k)] = Px_new[b * nP + k];
    if (Ax_new)
        for (int k = tid; k < nA; k += T) Ax_o[b * nnzA + (Ax_idx ? Ax_idx[k] : k)] = Ax_new[b * nA + k];
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
    bool moved = false;  // a row changed class: the workspace factor (ffresh) no longer fits
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
            moved = moved || p.ct[b * m + i] != t;
            p.ct[b * m + i] = t;
        }
    }
    bad = block_any<T>(bad, flag);
    moved = block_any<T>(moved, flag);
    if (tid == 0) {
        p.status[b] = MPCQP_UNSOLVED_;
        if (l_in || u_in) p.err[b] = bad ? 1 : 0;
        if (moved) p.ffresh[b] = 0;
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
        for (int e = p.acsr_ptr[i]; e < p.acsr_ptr[i + 1]; ++e) s += Ax[p.acsr_pos[e]] * x[p.acsr_col[e]];
        p.z[b * m + i] = s;
    }
}

// ------------------------------------------------------------ launchers --
// diagnostic A/B switches read once per process (environment variable set to "1")
static bool getenv_flag(const char* name) {
    const char* v = getenv(name);
    return v && v[0] == '1';
}
static size_t lds_setup_base(const KParams& p) {
    return sizeof(double) * ((size_t)p.nnzP + p.nnzA + 3 * (size_t)p.npad + 2 * (size_t)p.m + 64) + 16;
}
static bool setup_staged(const KParams& p) {
    return lds_setup_base(p) + sizeof(int) * (size_t)setup_span(p) <= 96 * 1024;
}
size_t lds_setup_bytes(const KParams& p) {
    return lds_setup_base(p) + (setup_staged(p) ? sizeof(int) * (size_t)setup_span(p) : 0);
}
// register-list setup (k_setup_r): one padded column and one row per thread, the
// instantiation's list lengths and values per thread cover the plan; 0 = none fits
static int setup_r_variant(const KParams& p) {
    if (p.npad > T || p.m > T || p.pk > 4) return 0;
    if (p.gk <= 6 && p.nnzA <= 2 * T && p.nnzP <= T) return 1;
    if (p.gk <= 8 && p.nnzA <= 3 * T && p.nnzP <= T) return 2;
    return 0;
}
// the wide one (k_setup_wide): 1 when it fits; the 512-thread form from kSetupHalfB instances
// (two per CU) -- fewer leave CUs idle, where the 1024-thread form's shorter latency wins
constexpr long kSetupHalfB = 512;
static int setup_rw_fits(const KParams& p) {
    return p.npad <= TWIDE && p.m <= TWIDE && p.pk <= 4 && p.gk <= 8 && p.nnzA <= 3 * TWIDE && p.nnzP <= TWIDE;
}

hipError_t launch_setup(const KParams& p, long B, const double* Px, const double* Ax, const double* q,
                        const double* l, const double* u, hipStream_t st, bool keep) {
    if (const int v = setup_r_variant(p); v && !getenv_flag("MPCQP_SETUP_STAGED")) {
        const size_t lds = lds_setup_r_bytes(p.nnzP, p.nnzA, p.npad, p.m);
        auto k = keep ? (v == 1 ? k_setup_r<6, 4, 2, 1, true> : k_setup_r<8, 4, 3, 1, true>)
                      : (v == 1 ? k_setup_r<6, 4, 2, 1, false> : k_setup_r<8, 4, 3, 1, false>);
        hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k, dim3((unsigned)B), dim3(T), lds, st, p, Px, Ax, q, l, u);
        return hipGetLastError();
    }
    if (setup_rw_fits(p) && !getenv_flag("MPCQP_SETUP_STAGED")) {
        // (the same columns / rows / values per workgroup either way: the fit is the same)
        const size_t lds = lds_setup_wide_bytes(p.nnzP, p.nnzA, p.npad, p.m, TWIDE);
        const bool half = B >= kSetupHalfB && !getenv_flag("MPCQP_SETUP_FULL");
        auto k = half ? (keep ? k_setup_wide<512, 2, 6, true> : k_setup_wide<512, 2, 6, false>)
                      : (keep ? k_setup_wide<TWIDE, 1, 3, true> : k_setup_wide<TWIDE, 1, 3, false>);
        hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k, dim3((unsigned)B), dim3(half ? 512 : TWIDE), lds, st, p, Px, Ax, q, l, u,
                           (const double*)nullptr, (const double*)nullptr);
        return hipGetLastError();
    }
    size_t lds = lds_setup_bytes(p);
    auto k = setup_staged(p) ? (keep ? k_setup<true, true> : k_setup<true, false>)
                             : (keep ? k_setup<false, true> : k_setup<false, false>);
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3((unsigned)B), dim3(T), lds, st, p, Px, Ax, q, l, u);
    return hipGetLastError();
}
hipError_t launch_update_mat(const KParams& p, long B, double* Px_io, double* Ax_io, double* q_io, double* l_io,
                             double* u_io, const double* Px_new, const int* Px_idx, int nP, const double* Ax_new,
                             const int* Ax_idx, int nA, hipStream_t st) {
    hipLaunchKernelGGL(k_unscale_mat, dim3((unsigned)B), dim3(T), 0, st, p, Px_io, Ax_io, q_io, l_io, u_io, Px_new,
                       Px_idx, nP, Ax_new, Ax_idx, nA);
    if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    return launch_setup(p, B, Px_io, Ax_io, q_io, l_io, u_io, st, true);
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
bool setup_warm_fused(const KParams& p) { return setup_rw_fits(p) && !getenv_flag("MPCQP_SETUP_STAGED"); }
hipError_t launch_setup_warm(const KParams& p, long B, const double* Px, const double* Ax, const double* q,
                             const double* l, const double* u, const double* x0, const double* y0, hipStream_t st) {
    if (!setup_warm_fused(p)) {
        if (hipError_t e = launch_setup(p, B, Px, Ax, q, l, u, st, false); e != hipSuccess) return e;
        return launch_warm(p, B, x0, y0, st);
    }
    const size_t lds = lds_setup_wide_bytes(p.nnzP, p.nnzA, p.npad, p.m, TWIDE);
    const bool half = B >= kSetupHalfB && !getenv_flag("MPCQP_SETUP_FULL");
    auto k = half ? k_setup_wide<512, 2, 6, false, true> : k_setup_wide<TWIDE, 1, 3, false, true>;
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3((unsigned)B), dim3(half ? 512 : TWIDE), lds, st, p, Px, Ax, q, l, u, x0, y0);
    return hipGetLastError();
}

__global__ void k_iota(int* __restrict__ order, long B) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < B) order[i] = (int)i;
}
__global__ __launch_bounds__(256) void k_gather(GatherList g, char* __restrict__ dst) {
    const long t0 = (long)blockIdx.x * 256 + threadIdx.x, stride = (long)gridDim.x * 256;
    for (int s = 0; s < g.nseg; ++s) {
        const GatherSeg& sg = g.seg[s];
        if (sg.sz == 8) {
            const double* src = (const double*)sg.src;
            double* d = (double*)(dst + sg.off);
            for (long i = t0; i < sg.cnt; i += stride) d[i] = src ? src[i] : 0.0;
        } else {
            const int* src = (const int*)sg.src;
            int* d = (int*)(dst + sg.off);
            for (long i = t0; i < sg.cnt; i += stride) d[i] = src ? src[i] : 0;
        }
    }
}

hipError_t launch_gather(const GatherList& g, void* dst, hipStream_t st) {
    if (g.nseg <= 0 || g.nseg > kGatherMax) return hipErrorInvalidValue;
    const long blocks = std::min<long>(std::max<long>((g.most + 255) / 256, 1), 1024);
    hipLaunchKernelGGL(k_gather, dim3((unsigned)blocks), dim3(256), 0, st, g, (char*)dst);
    return hipGetLastError();
}

hipError_t launch_iota(int* order, long B, hipStream_t st) {
    hipLaunchKernelGGL(k_iota, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, st, order, B);
    return hipGetLastError();
}

// ------------------------------------------------------------------ order --
// Dispatch order for the next solve on this workspace: longest previous solve first.
// A batch larger than the resident slots (cfg 2: 1024 instances, 512 two-wave
// workgroups at once) runs in rounds, and the kernel ends with its slowest instance;
// an instance that needs 350 ADMM iterations against a mean of 63 should start in
// the first round, not 200 us late.  Consecutive solves on one handle (the receding-
// horizon loop: update/setup, solve) see nearby problems, so the previous iteration
// count predicts the next.  The order only moves instances between workgroup slots:
// every instance's arithmetic, and so its result, is unchanged.
// One workgroup: counting sort on iter >> shift (descending), 256 bins.
constexpr int kOrderT = 1024, kOrderBins = 256;
// pred / odecay (KParams::pred): the key is max(iter, pred), and pred becomes key * odecay / 8.
__global__ __launch_bounds__(kOrderT) void k_order(const int* __restrict__ iter, int* __restrict__ order, long B,
                                                  int shift, int* __restrict__ pred, int odecay) {
    __shared__ int cnt[kOrderBins];
    const int t = threadIdx.x;
    if (t < kOrderBins) cnt[t] = 0;
    __syncthreads();
    auto key = [&](long i) { return odecay ? max(iter[i], pred[i]) : iter[i]; };
    auto bin = [&](long i) {
        const int k = key(i) >> shift;
        return kOrderBins - 1 - (k < kOrderBins - 1 ? k : kOrderBins - 1);
    };
    for (long i = t; i < B; i += kOrderT) atomicAdd(&cnt[bin(i)], 1);
    __syncthreads();
    if (t == 0) {
        int s = 0;
        for (int k = 0; k < kOrderBins; ++k) {
            const int c = cnt[k];
            cnt[k] = s;
            s += c;
        }
    }
    __syncthreads();
    for (long i = t; i < B; i += kOrderT) {
        order[atomicAdd(&cnt[bin(i)], 1)] = (int)i;
        if (odecay) pred[i] = (int)(((long)key(i) * odecay) >> 3);  // (only thread t reads / writes pred[i])
    }
}

hipError_t launch_order(const KParams& p, long B, hipStream_t st) {
    // a batch that fits the resident workgroup slots (CUs x the variant's occupancy,
    // api.hip::alloc_shard) starts all at once: the order cannot move anything
    if (!p.order || B <= p.slots) return hipSuccess;
    if (p.done && B <= kOrderFuseMax) return hipSuccess;  // sorted by the solve kernel's last workgroup
    int shift = 0;
    while ((p.max_iter >> shift) >= kOrderBins) ++shift;
    hipLaunchKernelGGL(k_order, dim3(1), dim3(kOrderT), 0, st, (const int*)p.iter, const_cast<int*>(p.order), B,
                       shift, p.odecay && p.pred ? p.pred : nullptr, p.odecay && p.pred ? p.odecay : 0);
    return hipGetLastError();
}
// Streaming copy (mpcqp_debug_copy, bench.py's achievable-HBM reference): each lane moves G
// 16-byte granules per pass, loads issued together ahead of the stores, grid-stride; NT:
// non-temporal loads and stores (no L2 / MALL pollution) or the default policy.
typedef double v2d __attribute__((ext_vector_type(2)));
template <bool NT, int G>
__global__ __launch_bounds__(256) void k_copy16(const v2d* __restrict__ s, v2d* __restrict__ d, long n2) {
    const long per = (long)G * 256;  // granules per workgroup pass
    for (long base = (long)blockIdx.x * per; base < n2; base += (long)gridDim.x * per) {
        const long i = base + threadIdx.x;
        v2d a[G];
#pragma unroll
        for (int k = 0; k < G; ++k) a[k] = NT ? __builtin_nontemporal_load(s + i + k * 256) : s[i + k * 256];
#pragma unroll
        for (int k = 0; k < G; ++k) {
            if (NT) __builtin_nontemporal_store(a[k], d + i + k * 256);
            else d[i + k * 256] = a[k];
        }
    }
}

// form: 0 non-temporal, 4 granules per lane, 2048 workgroups; 1 default policy, 4 granules,
// 2048; 2 default policy, 8 granules, 4096; 3 / 4 default policy / non-temporal, 4 granules, one
// pass (a workgroup per 16 KiB, no grid-stride loop) (n % 8192 == 0)
hipError_t launch_copy16(const double* src, double* dst, long n, hipStream_t st, int form) {
    const v2d* s = (const v2d*)src;
    v2d* d = (v2d*)dst;
    switch (form) {
        case 0: hipLaunchKernelGGL((k_copy16<true, 4>), dim3(2048), dim3(256), 0, st, s, d, n / 2); break;
        case 1: hipLaunchKernelGGL((k_copy16<false, 4>), dim3(2048), dim3(256), 0, st, s, d, n / 2); break;
        case 2: hipLaunchKernelGGL((k_copy16<false, 8>), dim3(4096), dim3(256), 0, st, s, d, n / 2); break;
        case 3: hipLaunchKernelGGL((k_copy16<false, 4>), dim3((unsigned)(n / 2048)), dim3(256), 0, st, s, d, n / 2); break;
        default: hipLaunchKernelGGL((k_copy16<true, 4>), dim3((unsigned)(n / 2048)), dim3(256), 0, st, s, d, n / 2); break;
    }
    return hipGetLastError();
}

}  // namespace mpcqp
