// solve_big.hip -- the ADMM kernel for long horizons (many factor blocks).
//
// Why a separate kernel: the 256-thread k_solve keeps the block-tridiagonal factor
// of K = P + sigma I + A' diag(rho) A in registers only up to 8 blocks; beyond that
// (NB = 0 instantiation) every ADMM iteration re-reads three 32 x 32 tiles per block
// from the per-instance workspace -- 3 * 17 * 8 KB = 408 KB per iteration at
// cfg 5 (N = 50, nb = 17), far more than an XCD's L2 holds for its resident
// instances, so the sweep ran at HBM speed (~55k cycles per iteration).
//
// Here one 512-thread workgroup (8 waves, two per SIMD) holds the whole factor on
// chip:
//   registers  S_k^{-1}[i][jl + 16 c] (c < 2) for every block k   (2 doubles / block)
//              H_k[i][jl] = F_{k+1}[jl][i]  (jl < amax <= 16)       (1 double / block)
//              with (i, jl) = (t / 16, t % 16): row i is summed by one 16-lane DPP row
//   LDS        F_k rows r < amax (the only nonzero rows: block k couples to block
//              k-1 through its first BFS level), amax x 32 per block
// and the sweep is
//   forward   k = 1..nb-1:  t_{k-1} = S_{k-1}^{-1} w_{k-1},  w_k -= F_k w_{k-1}   (1 barrier)
//             t_{nb-1} = S_{nb-1}^{-1} w_{nb-1}
//   backward  k = nb-2..0:  x_k = t_k - H_k x_{k+1}[0, amax)                     (1 barrier)
// -- the same elimination as solve.hip::bt_solve with the tiles on chip.
//
// Everything else (rhs gather, row update, termination checks, rho adaptation,
// refactorisation, unscaling) follows solve.hip's k_solve with 512 threads.
// Reference semantics: OSQP 0.6 osqp_solve (Control/MPC/mpc_dynamics.py:392-396 at
// N = 30 / 50); tests/test_gpu_parity.py and tests/test_mpc_device.py compare with
// the CPU oracle.
#include <hip/hip_runtime.h>

#include "solve_phases.h"

namespace mpcqp {

constexpr int TB = kThreadsBig;

template <int NBM>
struct BigFactor {
    double Si[NBM][2], H[NBM > 1 ? NBM - 1 : 1];
    // Sg: S_k^{-1} tiles, Fg: F_k tiles (rows < amax valid); F rows go to Fc (LDS)
    __device__ __forceinline__ void load(int nb, int amax, const double* __restrict__ Fg,
                                         const double* __restrict__ Sg, double* __restrict__ Fc) {
        const int tid = threadIdx.x, i = tid >> 4, jl = tid & 15;
#pragma unroll
        for (int k = 0; k < NBM; ++k) {
            if (k < nb) {
                Si[k][0] = Sg[(long)k * SS + i * S + jl];
                Si[k][1] = Sg[(long)k * SS + i * S + jl + 16];
            }
            if (k < NBM - 1) H[k] = (k + 1 < nb && jl < amax) ? Fg[(long)(k + 1) * SS + jl * S + i] : 0.0;
        }
        for (int o = tid; o < (nb - 1) * amax * S; o += TB) {
            const int k = o / (amax * S), r = o - k * amax * S;
            Fc[o] = Fg[(long)(k + 1) * SS + r];
        }
    }
};

// xt = K^{-1} rb (rb is overwritten by the forward sweep).  2 nb - 1 barriers.
template <int NBM>
__device__ __forceinline__ void big_solve(const BigFactor<NBM>& R, int nb, int amax, const double* Fc, double* rb,
                                          double* xt) {
    int opq = 0;
    asm volatile("" : "+s"(opq));  // keep per-block LDS addresses out of the register budget
    const int tid = threadIdx.x, i = tid >> 4, jl = (tid & 15) + opq;
    const bool frow = i < amax;
#pragma unroll
    for (int k = 1; k < NBM; ++k) {
        if (k < nb) {
            const double* v = rb + (k - 1) * S;
            const double v0 = v[jl], v1 = v[jl + 16];
            const double s2 = reduce16(R.Si[k - 1][0] * v0 + R.Si[k - 1][1] * v1);
            if (frow) {
                const double* f = Fc + ((k - 1) * amax + i) * S;
                const double s1 = reduce16(f[jl] * v0 + f[jl + 16] * v1);
                if ((tid & 15) == 0) rb[k * S + i] -= s1;
            }
            if ((tid & 15) == 0) xt[(k - 1) * S + i] = s2;
            __syncthreads();
        }
    }
#pragma unroll
    for (int k = 0; k < NBM; ++k) {
        if (k == nb - 1) {
            const double* v = rb + k * S;
            const double s2 = reduce16(R.Si[k][0] * v[jl] + R.Si[k][1] * v[jl + 16]);
            if ((tid & 15) == 0) xt[k * S + i] = s2;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = NBM - 2; k >= 0; --k) {
        if (k <= nb - 2) {
            const double s = reduce16(R.H[k] * xt[(k + 1) * S + (jl & 15)]);
            if ((tid & 15) == 0) xt[k * S + i] -= s;
            __syncthreads();
        }
    }
}

// LDS after the common carve (solve.hip::lds_solve_bytes): the F rows
__device__ __forceinline__ double* big_fc(const SLds& L) {
    const unsigned long a = ((unsigned long)(L.flag + 16) + 15ul) & ~15ul;
    return (double*)a;
}

template <int NBM, int K, int CS, int RS>
__global__ __launch_bounds__(TB, 1) void k_solve_b(KParams p, double* __restrict__ xo, double* __restrict__ yo,
                                                   int factor_only) {
    const int tid = threadIdx.x;
    const long b = blockIdx.x;
    const int n = p.n, m = p.m, npad = p.npad, nnzP = p.nnzP, nnzA = p.nnzA, nb = p.nb, amax = p.amax;
    SL2 C = carve(p);
    SLds& L = C.L;
    double* X = C.X;
    double* Z = C.Z;
    double* dY = C.dY;
    double* Fc = big_fc(L);
    const double* Fg = p.F + b * (long)nb * SS;
    const double* Sg = p.Si + b * (long)nb * SS;

    if (p.err[b]) {  // invalid data (flagged by setup/update): NaN outputs
        for (int j = tid; j < n; j += TB) if (xo) xo[b * n + j] = __builtin_nan("");
        for (int i = tid; i < m; i += TB) if (yo) yo[b * m + i] = __builtin_nan("");
        if (tid == 0) p.status[b] = MPCQP_NON_CVX_;
        return;
    }

#ifdef MPCQP_PHASE_PROF
    long long tph = 0, t0c = 0, t0w = 0;
    const bool prof = p.prof != nullptr;
    if (prof) { t0w = wall_clock64(); t0c = tph = clock64(); if (tid < 16) L.pacc[tid] = 0; }
#define PH(k) if (prof && tid == 0) { const long long t_ = clock64(); L.pacc[k] += t_ - tph; tph = t_; }
#else
#define PH(k)
#endif

    const double cval = p.scal[b * 4 + 0], cinv = p.scal[b * 4 + 1];
    double rho = p.scal[b * 4 + 2];
    const double sigma = p.sigma, alpha = p.alpha;
    const bool warm = p.warm_start != 0;
    for (int e = tid; e < nnzA; e += TB) L.Acsc[e] = p.Ax[b * nnzA + p.acsc_v[e]];
    if (tid == 0) L.Acsc[nnzA] = 0.0;  // the gather lists' padding slot
    for (int v = tid; v < nnzP; v += TB) L.Pv[v] = p.Px[b * nnzP + v];
    if (tid == 0) L.Pv[nnzP] = 0.0;
    for (int i = tid; i < m; i += TB) {
        L.lo[i] = p.l[b * m + i];
        L.up[i] = p.u[b * m + i];
        L.ct[i] = p.ct[b * m + i];
        Z[i] = warm ? p.z[b * m + i] : 0.0;
        dY[i] = 0.0;
    }
    for (int pc = tid; pc < npad; pc += TB) {
        L.qv[pc] = p.q[b * npad + pc];
        X[pc] = warm ? p.x[b * npad + pc] : 0.0;
    }
    if (tid < 16) L.res[tid] = 0.0;
    if (tid < 4) L.flag[tid] = 0;

    int status = MPCQP_UNSOLVED_, rho_updates = 0, iter = 0, info_iter = 0;
    bool can_check = false, need_factor = true;
    // y in registers for the whole solve (ys is its LDS copy for the out-of-line phases)
    double y[RS];
#pragma unroll
    for (int s = 0; s < RS; ++s) {
        const int i = tid + s * TB;
        y[s] = (i < m && warm) ? p.y[b * m + i] : 0.0;
    }
    PH(5)
    for (;;) {
        __syncthreads();
        if (need_factor) {  // start, and after a rho change
            need_factor = false;
            const bool ok = factorize_nl<TB>(p.self, b, rho);
            if (!ok) {
                if (iter == 0) {
                    for (int j = tid; j < n; j += TB) if (xo) xo[b * n + j] = __builtin_nan("");
                    for (int i = tid; i < m; i += TB) if (yo) yo[b * m + i] = __builtin_nan("");
                    if (tid == 0) p.status[b] = MPCQP_NON_CVX_;
                    return;
                }
                status = MPCQP_NON_CVX_;
                can_check = true;  // skip the final check_termination
                break;
            }
            if (factor_only) return;
            PH(0)
        }
        // ---- run state (re-derived at every run start; nothing but scalars lives across calls) ----
        BigFactor<NBM> RF;
        RF.load(nb, amax, Fg, Sg, Fc);
        int cvar[CS];
        Gather<K> cg[CS];
#pragma unroll
        for (int s = 0; s < CS; ++s) {
            const int pc = tid + s * TB;
            cvar[s] = pc < npad ? p.pad_var[pc] : -1;
            if (pc < npad) cg[s].load(p.gcol + (long)pc * kGS);
            else cg[s].clear(nnzA);
        }
        Gather<K> rg[RS];
#pragma unroll
        for (int s = 0; s < RS; ++s) {
            const int i = tid + s * TB;
            if (i < m) {
                rg[s].load(p.grow + (long)i * kGS);
                L.w[i] = rho_of(L.ct[i], rho) * Z[i] - y[s];  // w = rho z_prev - y (rho may be new)
            } else {
                rg[s].clear(nnzA);
            }
        }
        int stop_at = p.max_iter;
        if (p.check_term) stop_at = min(stop_at, (iter / p.check_term + 1) * p.check_term);
        if (p.adaptive_rho && p.rho_interval) stop_at = min(stop_at, (iter / p.rho_interval + 1) * p.rho_interval);
        __syncthreads();
        PH(5)
        const double r_hi = RHO_EQ_OVER_RHO_INEQ * rho;
        const double ri_lo = 1.0 / RHO_MIN, ri_mid = 1.0 / rho, ri_hi = 1.0 / r_hi;
        while (iter < stop_at) {
            ++iter;
            int opq = 0;
            asm volatile("" : "+s"(opq));
            const int tido = tid + opq;
            // rhs = sigma x_prev - q + A' (rho z_prev - y)
#pragma unroll
            for (int s = 0; s < CS; ++s) {
                const int pc = tido + s * TB;
                if (pc < npad)
                    L.rb[pc] = cvar[s] >= 0 ? (sigma * X[pc] - L.qv[pc]) + cg[s].dot(L.Acsc, L.w) : 0.0;
            }
            __syncthreads();
            PH(1)
            big_solve<NBM>(RF, nb, amax, Fc, L.rb, L.xt);
            PH(2)
            // z~ = A x~ ; relaxed + projected z ; y ; next w.   x update; deltas for the checks.
#pragma unroll
            for (int s = 0; s < RS; ++s) {
                const int i = tido + s * TB;
                if (i < m) {
                    const double zt = rg[s].dot(L.Acsc, L.xt);
                    const signed char cl = L.ct[i];
                    const double rv = cl < 0 ? RHO_MIN : (cl > 0 ? r_hi : rho);
                    const double rvi = cl < 0 ? ri_lo : (cl > 0 ? ri_hi : ri_mid);
                    const double zr = alpha * zt + (1.0 - alpha) * Z[i];
                    const double zn = cmin(cmax(zr + rvi * y[s], L.lo[i]), L.up[i]);
                    const double d = rv * (zr - zn);
                    Z[i] = zn;
                    dY[i] = d;
                    y[s] += d;
                    L.w[i] = rv * zn - y[s];
                }
            }
#pragma unroll
            for (int s = 0; s < CS; ++s) {
                const int pc = tido + s * TB;
                if (pc < npad) {
                    const double xold = X[pc];
                    const double xn = alpha * L.xt[pc] + (1.0 - alpha) * xold;
                    X[pc] = xn;
                    L.rb[pc] = xn - xold;
                }
            }
            __syncthreads();
            PH(3)
        }
#pragma unroll
        for (int s = 0; s < RS; ++s) { const int i = tid + s * TB; if (i < m) L.ys[i] = y[s]; }
        __syncthreads();
        // ---- out-of-line phases ----
        can_check = p.check_term && (iter % p.check_term == 0);
        const bool do_rho = p.adaptive_rho && p.rho_interval && (iter % p.rho_interval == 0);
        if (!can_check && !do_rho) break;  // max_iter reached
        update_info_nl<TB>(p.self, b, cinv);
        info_iter = iter;
        bool stop = false;
        if (can_check) {
            status = check_termination_nl<TB>(p.self, b, cval, cinv, 0);
            stop = status != MPCQP_UNSOLVED_;
        }
        if (!stop && do_rho) {
            Res R;
            R.restore(L.res);
            const double pr = R.rpri / (cmax(R.rz, R.rax) + DIVISION_TOL);
            const double du = R.rdua / (cmax(cmax(R.rq, R.raty), R.rpx) + DIVISION_TOL);
            double rn = rho * sqrt(pr / (du + DIVISION_TOL));
            rn = cmin(cmax(rn, RHO_MIN), RHO_MAX);
            if (rn > rho * p.rho_tol || rn < rho / p.rho_tol) {
                rho = cmin(cmax(rn, RHO_MIN), RHO_MAX);
                rho_updates++;
                need_factor = true;
            }
        }
        __syncthreads();
        PH(4)
        if (stop || iter >= p.max_iter) break;
    }
    if (!can_check && status == MPCQP_UNSOLVED_) {
        update_info_nl<TB>(p.self, b, cinv);
        info_iter = iter;
        status = check_termination_nl<TB>(p.self, b, cval, cinv, 0);
    }
    const bool has_sol = !(status == MPCQP_PRIMAL_INFEASIBLE_ || status == MPCQP_PRIMAL_INFEASIBLE_INACCURATE_ ||
                           status == MPCQP_DUAL_INFEASIBLE_ || status == MPCQP_DUAL_INFEASIBLE_INACCURATE_ ||
                           status == MPCQP_NON_CVX_);
    if (has_sol) objective_nl<TB>(p.self, cinv);
    if (status == MPCQP_UNSOLVED_) {
        status = check_termination_nl<TB>(p.self, b, cval, cinv, 1);
        if (status == MPCQP_UNSOLVED_) status = MPCQP_MAX_ITER_REACHED_;
    }
    finalize_nl<TB>(p.self, b, xo, yo, cinv, rho, status, info_iter, rho_updates);
#ifdef MPCQP_PHASE_PROF
    if (prof) {
        __syncthreads();
        PH(5)
        if (tid == 0) {
#pragma unroll
            for (int k = 0; k < 6; ++k) p.prof[b * kProfSlots + k] = L.pacc[k];
#pragma unroll
            for (int k = 8; k < 12; ++k) p.prof[b * kProfSlots + k] = L.pacc[k];
            p.prof[b * kProfSlots + 6] = clock64() - t0c;
            p.prof[b * kProfSlots + 7] = wall_clock64() - t0w;
        }
    }
#endif
#undef PH
}

size_t lds_solve_bytes_big(const KParams& p) {
    return lds_solve_bytes(p) + 16 + sizeof(double) * (size_t)(p.nb - 1) * p.amax * S;
}

template <int NBM, int K, int CS, int RS>
static hipError_t go_b(const KParams& p, long B, double* xo, double* yo, int fo, hipStream_t st) {
    const size_t lds = lds_solve_bytes_big(p);
    auto k = k_solve_b<NBM, K, CS, RS>;
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3((unsigned)B), dim3(TB), lds, st, p, xo, yo, fo);
    return hipGetLastError();
}

hipError_t launch_solve_big(const KParams& p, long B, double* xo, double* yo, int factor_only, hipStream_t st) {
    switch (p.variant) {
        case 11: return go_b<12, 8, 1, 2>(p, B, xo, yo, factor_only, st);
        case 12: return go_b<18, 8, 2, 2>(p, B, xo, yo, factor_only, st);
        case 13: return go_b<24, 8, 2, 3>(p, B, xo, yo, factor_only, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace mpcqp
