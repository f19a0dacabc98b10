// solve.hip -- the ADMM kernel (osqp_solve restated for MI355X / gfx950).
//
// One 256-thread workgroup (4 wavefronts) per QP instance, persistent over the
// whole solve.  Work decomposition inside the workgroup:
//   * thread t owns padded variables  pc = t + 256*s  (s < CS) and constraint
//     rows  i = t + 256*s  (s < RS): x, x_prev, z, z_prev, y and delta_y live in
//     its registers for the whole solve, with its row / column gather lists
//     (<= KMAX entries, 16-bit indices) -- no global-memory traffic per iteration;
//   * A is kept in LDS twice (padded-CSC order for A'w, CSR order for A x~);
//   * the block-tridiagonal factor of K = P + sigma I + A' diag(rho) A (plan.h)
//     is distributed over the 256 threads' registers when it has NB <= 16
//     blocks of 32: thread (i = t/8, jg = t%8) holds elements [i][jg+8c],
//     c < 4, of every F_k, H_k = F_{k+1}', S_k^{-1} tile; row sums of the tile
//     mat-vecs use three DPP steps inside an 8-lane half-row.  Larger plans
//     (NB = 0 instantiation) read the tiles from the per-instance workspace.
// Per ADMM iteration: 2*nb + 1 workgroup barriers.
//
// Reference semantics: osqp_solve / update_xz_tilde / update_x / update_z /
// update_y / update_info / check_termination / adapt_rho / store_solution of
// OSQP 0.6 (the solver behind vehicle_lateral_mpc_slack_increment.py:248 and
// Control/MPC/mpc_dynamics.py:396); oracle/osqp_oracle.c restates the same
// algorithm on the CPU and tests/test_gpu_parity.py compares the two.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "solve_phases.h"

namespace mpcqp {


// Register-resident factor.  F_k = E_k S_{k-1}^{-1} is nonzero only in the rows of
// block k that couple to block k-1 (its first BFS level, local rows < A), and
// H_{k-1} = F_k' only in those columns, so each thread keeps
//   Si[k][4]  : S_k^{-1}[i][jg+8c],          (i, jg) = (t/8, t%8)
//   F[k][A/8] : F_{k+1}[r][j],  A = 8 : (r, j) = (t/32, t%32);  A = 16: (t/16, t%16 + 16c)
//   H[k][A/8] : H_k[i][jg+8c],  c < A/8
// (A = 32 keeps the full tiles in the Si layout).
template <int NB, int A>
struct RegFactor {
    static constexpr int NF = A == 32 ? 4 : A / 8;
    double F[NB > 1 ? NB - 1 : 1][NF], H[NB > 1 ? NB - 1 : 1][NF], Si[NB > 0 ? NB : 1][4];
    __device__ __forceinline__ void load(int nb, const double* Fg, const double* Hg, const double* Sg) {
        const int tid = threadIdx.x, i = tid >> 3, jg = tid & 7;
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            if (k < nb) {
#pragma unroll
                for (int c = 0; c < 4; ++c) Si[k][c] = Sg[(long)k * SS + i * S + jg + 8 * c];
            }
            if (k + 1 < nb && k < NB - 1) {
                const double* Fk = Fg + (long)(k + 1) * SS;
#pragma unroll
                for (int c = 0; c < NF; ++c) {
                    if constexpr (A == 8) F[k][c] = Fk[(tid >> 5) * S + (tid & 31)];
                    else if constexpr (A == 16) F[k][c] = Fk[(tid >> 4) * S + (tid & 15) + 16 * c];
                    else F[k][c] = Fk[i * S + jg + 8 * c];
                    H[k][c] = Fk[(jg + 8 * c) * S + i];  // H_k = F_{k+1}'
                }
            }
        }
    }
};

template <int N>
__device__ __forceinline__ double dotn(const double (&a)[N], const double* v, int jg) {
    double acc = a[0] * v[jg];
#pragma unroll
    for (int c = 1; c < N; ++c) acc += a[c] * v[jg + 8 * c];
    return acc;
}
__device__ __forceinline__ double dot4(const double (&a)[4], const double* v, int jg) {
    return (a[0] * v[jg] + a[1] * v[jg + 8]) + (a[2] * v[jg + 16] + a[3] * v[jg + 24]);
}
__device__ __forceinline__ double dot4g(const double* a, const double* v, int jg) {
    return (a[jg] * v[jg] + a[jg + 8] * v[jg + 8]) + (a[jg + 16] * v[jg + 16] + a[jg + 24] * v[jg + 24]);
}

// xt = K^{-1} rb (rb is overwritten by the forward sweep).  2*nb - 1 barriers.
template <int NB, int A>
__device__ __forceinline__ void bt_solve(const KParams& p, const RegFactor<NB, A>& R, const double* Fg,
                                         const double* Hg, const double* Sg, double* rb, double* xt) {
    int opq = 0;
    asm volatile("" : "+s"(opq));  // keep per-block LDS addresses out of the register budget
    const int tid = threadIdx.x, i = tid >> 3, jg = (tid & 7) + opq;
    const int nb = NB > 0 ? NB : p.nb;  // register variants are instantiated for their exact block count
    if constexpr (NB > 0) {
        // forward sweep w_k -= F_k w_{k-1}, fused with t_{k-1} = S_{k-1}^{-1} w_{k-1}
#pragma unroll
        for (int k = 1; k < NB; ++k) {
            if (k < nb) {
                const double* v = rb + (k - 1) * S;
                const double s2 = reduce8(dot4(R.Si[k - 1], v, jg));
                if constexpr (A == 8) {
                    const int j = (tid & 31) + opq;
                    const double s1 = reduce32_hi(R.F[k - 1][0] * v[j]);
                    if ((tid & 31) == 31) rb[k * S + (tid >> 5)] -= s1;
                } else if constexpr (A == 16) {
                    const int j = (tid & 15) + opq;
                    const double s1 = reduce16(R.F[k - 1][0] * v[j] + R.F[k - 1][1] * v[j + 16]);
                    if ((tid & 15) == 0) rb[k * S + (tid >> 4)] -= s1;
                } else {
                    const double s1 = reduce8(dot4(R.F[k - 1], v, jg));
                    if (jg == 0) rb[k * S + i] -= s1;
                }
                if ((tid & 7) == 0) xt[(k - 1) * S + i] = s2;
                __syncthreads();
            }
        }
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            if (k == nb - 1) {
                const double s2 = reduce8(dot4(R.Si[k], rb + k * S, jg));
                if ((tid & 7) == 0) xt[k * S + i] = s2;
            }
        }
        __syncthreads();
        // backward sweep x_k = t_k - H_k x_{k+1}  (H_k reads only x_{k+1}[0, A))
#pragma unroll
        for (int k = NB - 2; k >= 0; --k) {
            if (k <= nb - 2) {
                const double s = reduce8(dotn(R.H[k], xt + (k + 1) * S, jg));
                if ((tid & 7) == 0) xt[k * S + i] -= s;
                __syncthreads();
            }
        }
    } else {
        for (int k = 1; k < nb; ++k) {
            const double* v = rb + (k - 1) * S;
            const double s1 = reduce8(dot4g(Fg + (long)k * SS + i * S, v, jg));
            const double s2 = reduce8(dot4g(Sg + (long)(k - 1) * SS + i * S, v, jg));
            if ((tid & 7) == 0) { rb[k * S + i] -= s1; xt[(k - 1) * S + i] = s2; }
            __syncthreads();
        }
        {
            const double s2 = reduce8(dot4g(Sg + (long)(nb - 1) * SS + i * S, rb + (nb - 1) * S, jg));
            if ((tid & 7) == 0) xt[(nb - 1) * S + i] = s2;
        }
        __syncthreads();
        for (int k = nb - 2; k >= 0; --k) {
            const double s = reduce8(dot4g(Hg + (long)k * SS + i * S, xt + (k + 1) * S, jg));
            if ((tid & 7) == 0) xt[k * S + i] -= s;
            __syncthreads();
        }
    }
}

// Three-phase solve (mode 2, NB <= 4):  K^{-1} = L^{-T} D^{-1} L^{-1}  with the
// blocks of L^{-1} precomputed (G_kj, factorize), so that x~ = K^{-1} b takes three
// parallel phases instead of a 2*nb-1 step sweep:
//   A: c_k = sum_{j<k} G_kj b_j          (rows < amax of block k)
//   B: t_k = S_k^{-1} (b_k + c_k)
//   C: x_k = t_k + sum_{j>k} G_jk' t_j
// Thread layouts:  Si as RegFactor;  GL[pair][e] = G_kj[r][c] with r = t / LPR,
// c = t % LPR + LPR e (LPR = 256 / A lanes per row);  GU[pair][e] = G_jk[r][i] with
// i = t / 8, r = t % 8 + 8 e.
template <int NB, int A>
struct RegFactor3 {
    static_assert(NB * 64 <= T, "one wave per diagonal block");
    static constexpr int NP = NB * (NB - 1) / 2 > 0 ? NB * (NB - 1) / 2 : 1;
    static constexpr int LPR = T / A;
    static constexpr int EL = A / 8;
    // Sw: wave w owns block w: thread t keeps S_w^{-1}[i][16 h + c], i = (t/2) % 32, h = t % 2
    double Sw[16], GL[NP][EL], GU[NP][EL];
    __device__ __forceinline__ void load(int amax, const double* Gg, const double* Sg) {
        const int tid = threadIdx.x, i = tid >> 3, jg = tid & 7;
        const long gs = (long)amax * S;
        {
            const int kb = tid >> 6, ib = (tid >> 1) & (S - 1), hb = tid & 1;
#pragma unroll
            for (int c = 0; c < 16; ++c) Sw[c] = kb < NB ? Sg[(long)kb * SS + ib * S + 16 * hb + c] : 0.0;
        }
        const int r = tid / LPR;
#pragma unroll
        for (int q = 0; q < NB * (NB - 1) / 2; ++q)
#pragma unroll
            for (int e = 0; e < EL; ++e) {
                const int c = tid % LPR + LPR * e, ru = jg + 8 * e;
                GL[q][e] = r < amax ? Gg[q * gs + r * S + c] : 0.0;
                GU[q][e] = ru < amax ? Gg[q * gs + ru * S + i] : 0.0;
            }
    }
};

// reduction over the LPR lanes of one G row (A = 8: 32 lanes, result in the upper 16)
template <int A>
__device__ __forceinline__ double reduce_lpr(double v) {
    if constexpr (A == 8) return reduce32_hi(v);
    else if constexpr (A == 16) return reduce16(v);
    else return reduce8(v);
}
template <int A>
__device__ __forceinline__ bool lpr_writer(int tid) {
    if constexpr (A == 8) return (tid & 31) == 31;
    else if constexpr (A == 16) return (tid & 15) == 0;
    else return (tid & 7) == 0;
}

// b in rb on entry; x~ in rb on exit (t in xt, corrections in cor).  3 barriers.
template <int NB, int A>
__device__ __forceinline__ void tri_solve(const RegFactor3<NB, A>& R, double* rb, double* xt, double* cor) {
    int opq = 0;
    asm volatile("" : "+s"(opq));
    const int tid = threadIdx.x, i = tid >> 3, jg = (tid & 7) + opq;
    constexpr int LPR = RegFactor3<NB, A>::LPR, EL = RegFactor3<NB, A>::EL;
    // A
    {
        const int r = tid / LPR, c0 = tid % LPR + opq;
#pragma unroll
        for (int k = 1; k < NB; ++k) {
            double acc = 0.0;
#pragma unroll
            for (int j = 0; j < k; ++j)
#pragma unroll
                for (int e = 0; e < EL; ++e) acc += R.GL[k * (k - 1) / 2 + j][e] * rb[j * S + c0 + LPR * e];
            const double sacc = reduce_lpr<A>(acc);
            if (lpr_writer<A>(tid)) cor[k * S + r] = sacc;
        }
    }
    __syncthreads();
    // B: wave k computes t_k; lanes (2i, 2i+1) split row i in halves (one DPP step)
    {
        const int kb = tid >> 6, ib = (tid >> 1) & (S - 1), hb = tid & 1;
        const double* wk = rb + kb * S + 16 * hb + opq;
        const double* ck = cor + kb * S + 16 * hb + opq;
        double a[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            double v0 = wk[4 * q], v1 = wk[4 * q + 1], v2 = wk[4 * q + 2], v3 = wk[4 * q + 3];
            if (4 * q < A && kb > 0 && hb == 0) {
                v0 += ck[4 * q]; v1 += ck[4 * q + 1]; v2 += ck[4 * q + 2]; v3 += ck[4 * q + 3];
            }
            a[q] = (R.Sw[4 * q] * v0 + R.Sw[4 * q + 1] * v1) + (R.Sw[4 * q + 2] * v2 + R.Sw[4 * q + 3] * v3);
        }
        double sacc = (a[0] + a[1]) + (a[2] + a[3]);
        sacc += dpp<0xB1>(sacc);
        if (kb < NB && hb == 0) xt[kb * S + ib] = sacc;
    }
    __syncthreads();
    // C
#pragma unroll
    for (int k = 0; k < NB; ++k) {
        double acc = 0.0;
#pragma unroll
        for (int j = k + 1; j < NB; ++j)
#pragma unroll
            for (int e = 0; e < EL; ++e) acc += R.GU[j * (j - 1) / 2 + k][e] * xt[j * S + jg + 8 * e];
        const double sacc = k + 1 < NB ? reduce8(acc) : 0.0;
        if ((tid & 7) == 0) rb[k * S + i] = xt[k * S + i] + sacc;
    }
    __syncthreads();
}

template <int NB, int A, int K, int CS, int RS, int W, bool TRI>
__global__ __launch_bounds__(T, W) void k_solve(KParams p, double* __restrict__ xo, double* __restrict__ yo,
                                                int factor_only) {
    const int tid = threadIdx.x;
    const long b = instance_of(p);
    const int n = p.n, m = p.m, npad = p.npad, nnzP = p.nnzP, nnzA = p.nnzA;
    SL2 C = carve(p);
    SLds& L = C.L;
    double* X = C.X;
    double* Z = C.Z;
    double* dY = C.dY;
    const double* Fg = p.F + b * (long)p.nb * SS;
    const double* Hg = p.H + b * (long)p.nb * SS;
    const double* Sg = p.Si + b * (long)p.nb * SS;
    // TRI: three-phase solve (x~ lands in rb, delta x goes to xt); else the sweep (x~ in xt, delta x in rb)
    static_assert(!TRI || (NB > 0 && NB <= 4), "three-phase solve needs a register factor of <= 4 blocks");
    double* const XT = TRI ? L.rb : L.xt;
    double* const DX = TRI ? L.xt : L.rb;

    if (p.err[b]) {  // invalid data (flagged by setup/update): NaN outputs
        for (int j = tid; j < n; j += T) if (xo) xo[b * n + j] = __builtin_nan("");
        for (int i = tid; i < m; i += T) if (yo) yo[b * m + i] = __builtin_nan("");
        if (tid == 0) fail_status(p, b);
        return;
    }

    // optional phase timers (thread 0's shader clock; every phase ends at a barrier)
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
    for (int e = tid; e < nnzA; e += T) L.Acsc[e] = p.Ax[b * nnzA + e];
    if (tid == 0) L.Acsc[nnzA] = 0.0;  // the gather lists' padding slot
    for (int v = tid; v < nnzP; v += T) L.Pv[v] = p.Px[b * nnzP + v];
    if (tid == 0) L.Pv[nnzP] = 0.0;
    for (int i = tid; i < m; i += T) {
        L.lo[i] = p.l[b * m + i];
        L.up[i] = p.u[b * m + i];
        L.ct[i] = p.ct[b * m + i];
        Z[i] = warm ? p.z[b * m + i] : 0.0;
        dY[i] = 0.0;
    }
    for (int pc = tid; pc < npad; pc += T) {
        L.qv[pc] = p.q[b * npad + pc];
        X[pc] = warm ? p.x[b * npad + pc] : 0.0;
    }
    if (tid < 16) L.res[tid] = 0.0;
    if (tid < 4) L.flag[tid] = 0;

    int status = MPCQP_UNSOLVED_, rho_updates = 0, iter = 0, info_iter = 0;
    bool can_check = false, need_factor = true;
    // y stays in registers for the whole solve (ys is its LDS copy for the
    // out-of-line phases; the factorisation scratch overwrites ys)
    double y[RS];
#pragma unroll
    for (int s = 0; s < RS; ++s) {
        const int i = tid + s * T;
        y[s] = (i < m && warm) ? p.y[b * m + i] : 0.0;
    }
    PH(5)
    // The solve alternates "runs" of ADMM iterations up to the next termination /
    // rho-adaptation point (no calls, everything in registers and LDS) with the
    // out-of-line phases.  The per-thread run state (factor tiles, gather lists)
    // is re-derived at the start of every run, so it is not live across a call
    // (the calling convention would otherwise spill it to scratch).
    for (;;) {
        __syncthreads();
        if (need_factor) {  // start, and after a rho change
            need_factor = false;
            const bool ok = factorize_nl<T>(p.self, b, rho);
            if (!ok) {
                if (iter == 0) {
                    for (int j = tid; j < n; j += T) if (xo) xo[b * n + j] = __builtin_nan("");
                    for (int i = tid; i < m; i += T) if (yo) yo[b * m + i] = __builtin_nan("");
                    if (tid == 0) fail_status(p, b);
                    return;
                }
                status = MPCQP_NON_CVX_;
                can_check = true;  // skip the final check_termination
                break;
            }
            if (factor_only) return;
            PH(0)
        }
        // ---- run state ----
        std::conditional_t<TRI, RegFactor3<NB, A>, RegFactor<NB, A>> RF;
        if constexpr (TRI) RF.load(p.amax, Hg, Sg);
        else if constexpr (NB > 0) RF.load(NB, Fg, Hg, Sg);
        int cvar[CS];
        Gather<K> cg[CS];
#pragma unroll
        for (int s = 0; s < CS; ++s) {
            const int pc = tid + s * T;
            cvar[s] = pc < npad ? p.pad_var[pc] : -1;
            if (pc < npad) cg[s].load(p.gcol + pc, &p.self->npad);
            else cg[s].clear(nnzA);
        }
        Gather<K> rg[RS];
#pragma unroll
        for (int s = 0; s < RS; ++s) {
            const int i = tid + s * T;
            if (i < m) {
                rg[s].load(p.grow + i, &p.self->m);
                L.w[i] = rho_of(L.ct[i], rho) * Z[i] - y[s];  // w = rho z_prev - y (rho may be new)
            } else {
                rg[s].clear(nnzA);
            }
        }
        // the run ends at the next termination check / rho adaptation / max_iter
        int stop_at = p.max_iter;
        if (p.check_term) stop_at = min(stop_at, (iter / p.check_term + 1) * p.check_term);
        if (p.adaptive_rho && p.rho_interval) stop_at = min(stop_at, (iter / p.rho_interval + 1) * p.rho_interval);
        __syncthreads();
        PH(5)
        // rho_vec / rho_inv_vec of the three row classes (OSQP keeps 1/rho_i precomputed)
        const double r_hi = RHO_EQ_OVER_RHO_INEQ * rho;
        const double ri_lo = 1.0 / RHO_MIN, ri_mid = 1.0 / rho, ri_hi = 1.0 / r_hi;
        while (iter < stop_at) {
            ++iter;
            // an opaque zero keeps per-thread LDS addresses out of the register budget
            int opq = 0;
            asm volatile("" : "+s"(opq));
            const int tido = tid + opq;
            // rhs = sigma x_prev - q + A' (rho z_prev - y)
#pragma unroll
            for (int s = 0; s < CS; ++s) {
                const int pc = tido + s * T;
                if (pc < npad)
                    L.rb[pc] = cvar[s] >= 0 ? (sigma * X[pc] - L.qv[pc]) + cg[s].dot(L.Acsc, L.w) : 0.0;
            }
            __syncthreads();
            PH(1)
            if constexpr (TRI) tri_solve<NB, A>(RF, L.rb, L.xt, L.cor);
            else bt_solve<NB, A>(p, RF, Fg, Hg, Sg, L.rb, L.xt);
            PH(2)
            // z~ = A x~ ; relaxed + projected z ; y ; next w.   x update; deltas for the checks.
#pragma unroll
            for (int s = 0; s < RS; ++s) {
                const int i = tido + s * T;
                if (i < m) {
                    const double zt = rg[s].dot(L.Acsc, XT);
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
                const int pc = tido + s * T;
                if (pc < npad) {
                    const double xold = X[pc];
                    const double xn = alpha * XT[pc] + (1.0 - alpha) * xold;
                    X[pc] = xn;
                    DX[pc] = xn - xold;
                }
            }
            __syncthreads();
            PH(3)
        }
#pragma unroll
        for (int s = 0; s < RS; ++s) { const int i = tid + s * T; if (i < m) L.ys[i] = y[s]; }
        __syncthreads();
        // ---- out-of-line phases (only scalars live across these calls) ----
        can_check = p.check_term && (iter % p.check_term == 0);
        const bool do_rho = p.adaptive_rho && p.rho_interval && (iter % p.rho_interval == 0);
        if (!can_check && !do_rho) break;  // max_iter reached
        update_info_nl<T>(p.self, b, cinv);
        info_iter = iter;
        bool stop = false;
        if (can_check) {
            status = check_termination_nl<T>(p.self, b, cval, cinv, 0);
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
        __syncthreads();  // red / res reused
        PH(4)
        if (stop || iter >= p.max_iter) break;
    }
    // ys holds y here
    if (!can_check && status == MPCQP_UNSOLVED_) {
        update_info_nl<T>(p.self, b, cinv);
        info_iter = iter;
        status = check_termination_nl<T>(p.self, b, cval, cinv, 0);
    }
    const bool has_sol = !(status == MPCQP_PRIMAL_INFEASIBLE_ || status == MPCQP_PRIMAL_INFEASIBLE_INACCURATE_ ||
                           status == MPCQP_DUAL_INFEASIBLE_ || status == MPCQP_DUAL_INFEASIBLE_INACCURATE_ ||
                           status == MPCQP_NON_CVX_);
    if (has_sol) objective_nl<T>(p.self, cinv);
    if (status == MPCQP_UNSOLVED_) {
        status = check_termination_nl<T>(p.self, b, cval, cinv, 1);
        if (status == MPCQP_UNSOLVED_) status = MPCQP_MAX_ITER_REACHED_;
    }
    finalize_nl<T>(p.self, b, xo, yo, cinv, rho, status, info_iter, rho_updates, p.ostat, p.oiter);
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

// ------------------------------------------------------------------ polish --
// OSQP 0.6 polish.c on the device, after the solve, on the scaled data (osqp_solve
// calls polish() when settings.polish and the status is "solved"; the reference
// never enables it -- SURVEY.md §8f F4, API parity).  The reduced KKT system
//   [[P + delta I, Ared'], [Ared, -delta I]] [x; y_red] = [-q; b_red]
// (Ared: the rows guessed active at the ADMM point -- lower-active z - l < -y,
// upper-active u - z < y, a row active at both ends appears twice; b_red their
// active bounds) is solved in its eliminated form
//   (P + delta I + Ared' Ared / delta) x = -q + Ared' b_red / delta,
//   y_red = (Ared x - b_red) / delta,
// which has the block-tridiagonal structure of the ADMM system (factorize<POL>).
// Iterative refinement against the unregularised matrix (polish_refine_iter steps)
// removes the delta error as OSQP's does.  Then y from y_red, the normal-cone
// projection of (A x, y), the residuals and OSQP's acceptance test; outputs, the
// warm-start iterates and the info are replaced only when the polished point is
// accepted.  pstat: 0 not run (status not solved), 1 accepted, -1 rejected.

// x~ = K_pol^{-1} rb (rb overwritten) with the mode-1 factor in the workspace:
// F_k rows < amax, S_k^{-1}.  Block Thomas, 2 nb - 1 barriers.
__device__ void pol_solve(const KParams& p, const double* __restrict__ Fg, const double* __restrict__ Sg,
                          double* rb, double* xt) {
    const int tid = threadIdx.x, i = tid >> 3, jg = tid & 7, nb = p.nb, amax = p.amax;
    for (int k = 0; k < nb; ++k) {
        const double* v = rb + k * S;
        const double* Sk = Sg + (long)k * SS + i * S;
        double a = 0.0;
#pragma unroll
        for (int c = 0; c < 4; ++c) a += Sk[jg + 8 * c] * v[jg + 8 * c];
        const double t = reduce8(a);
        if (k + 1 < nb && i < amax) {
            const double* Fk = Fg + (long)(k + 1) * SS + i * S;
            double f = 0.0;
#pragma unroll
            for (int c = 0; c < 4; ++c) f += Fk[jg + 8 * c] * v[jg + 8 * c];
            f = reduce8(f);
            if (jg == 0) rb[(k + 1) * S + i] -= f;
        }
        if (jg == 0) xt[k * S + i] = t;
        __syncthreads();
    }
    for (int k = nb - 2; k >= 0; --k) {  // x_k = t_k - F_{k+1}' x_{k+1}[0, amax)
        const double* F1 = Fg + (long)(k + 1) * SS;
        double a = 0.0;
        for (int r = jg; r < amax; r += 8) a += F1[r * S + i] * xt[(k + 1) * S + r];
        a = reduce8(a);
        if (jg == 0) xt[k * S + i] -= a;
        __syncthreads();
    }
}

__global__ __launch_bounds__(T) void k_polish(KParams p, double* __restrict__ xo, double* __restrict__ yo) {
    const int tid = threadIdx.x;
    const long b = blockIdx.x;
    const int n = p.n, m = p.m, npad = p.npad, nnzP = p.nnzP, nnzA = p.nnzA;
    if (p.status[b] != MPCQP_SOLVED_) {
        if (tid == 0) p.pstat[b] = 0;
        return;
    }
    SL2 C = carve(p);
    SLds& L = C.L;
    double* X = C.X;   // polish x
    double* YL = C.Z;  // duals of the lower-active copies
    double* AX = C.dY;
    const double cinv = p.scal[b * 4 + 1], idelta = 1.0 / p.delta;
    const double* Fg = p.F + b * (long)p.nb * SS;
    const double* Sg = p.Si + b * (long)p.nb * SS;
    for (int e = tid; e < nnzA; e += T) L.Acsc[e] = p.Ax[b * nnzA + e];
    if (tid == 0) L.Acsc[nnzA] = 0.0;
    for (int v = tid; v < nnzP; v += T) L.Pv[v] = p.Px[b * nnzP + v];
    if (tid == 0) L.Pv[nnzP] = 0.0;
    for (int i = tid; i < m; i += T) {  // form_Ared: the active-set guess
        const double lo = p.l[b * m + i], up = p.u[b * m + i], z = p.z[b * m + i], y = p.y[b * m + i];
        L.lo[i] = lo;
        L.up[i] = up;
        L.ct[i] = (signed char)((z - lo < -y ? 1 : 0) | (up - z < y ? 2 : 0));
    }
    for (int pc = tid; pc < npad; pc += T) L.qv[pc] = p.q[b * npad + pc];
    if (tid == 0) p.ffresh[b] = 0;  // the polish system's factor takes the workspace tiles
    __syncthreads();
    const bool ok = factorize_pol_nl<T>(p.self, b);
    if (!ok) {  // the reduced KKT matrix is not quasi-definite: polish fails
        if (tid == 0) p.pstat[b] = -1;
        return;
    }
    double* YU = L.ys;  // duals of the upper-active copies (V is free after the factorisation)
    for (int pc = tid; pc < npad; pc += T) X[pc] = 0.0;
    for (int i = tid; i < m; i += T) { YL[i] = 0.0; YU[i] = 0.0; }
    __syncthreads();
    for (int it = 0; it <= p.refine_iter; ++it) {
        // residual of [[P, Ared'], [Ared, 0]] [x; y_red] = [-q; b_red], folded into the
        // eliminated rhs: r_x + Ared' r_y / delta
        for (int i = tid; i < m; i += T) {
            const int fl = L.ct[i];
            const double ax = row_dot(p, L.Acsc, X, i);
            AX[i] = ax;
            const double rl = L.lo[i] - ax, ru = L.up[i] - ax;
            L.w[i] = ((fl & 1) ? rl * idelta - YL[i] : 0.0) + ((fl & 2) ? ru * idelta - YU[i] : 0.0);
        }
        __syncthreads();
        for (int pc = tid; pc < npad; pc += T)
            L.rb[pc] = p.pad_var[pc] >= 0 ? (-L.qv[pc] - psym_dot(p, L.Pv, X, pc)) + col_dot(p, L.Acsc, L.w, pc)
                                          : 0.0;
        __syncthreads();
        pol_solve(p, Fg, Sg, L.rb, L.xt);
        for (int i = tid; i < m; i += T) {  // dy = (Ared dx - r_y) / delta
            const int fl = L.ct[i];
            if (!fl) continue;
            const double adx = row_dot(p, L.Acsc, L.xt, i), ax = AX[i];
            if (fl & 1) YL[i] += (adx - (L.lo[i] - ax)) * idelta;
            if (fl & 2) YU[i] += (adx - (L.up[i] - ax)) * idelta;
        }
        __syncthreads();
        for (int pc = tid; pc < npad; pc += T) X[pc] += L.xt[pc];
        __syncthreads();
    }
    // polished (x, z, y): y from y_red (lower copy first, as get_ypol_from_yred),
    // then project_normalcone; residuals as update_info(polish = 1)
    const double* Eg = p.E + b * m;
    const double* Dg = p.D + b * npad;
    const bool unscaled = p.scaling && !p.scaled_term;
    double nrm[2] = {0.0, 0.0};
    double* Zp = AX;     // polished z
    double* Yp = L.w;    // polished y
    for (int i = tid; i < m; i += T) {
        const int fl = L.ct[i];
        const double ax = row_dot(p, L.Acsc, X, i);
        const double yv = (fl & 1) ? YL[i] : ((fl & 2) ? YU[i] : 0.0);
        const double t = ax + yv;
        const double zn = cmin(cmax(t, L.lo[i]), L.up[i]);
        Zp[i] = zn;
        Yp[i] = t - zn;
        const double pr = ax - zn;
        nrm[0] = cmax(nrm[0], fabs(unscaled ? pr / Eg[i] : pr));
    }
    __syncthreads();
    double obj[1] = {0.0};
    for (int pc = tid; pc < npad; pc += T) {
        if (p.pad_var[pc] < 0) continue;
        const double px = psym_dot(p, L.Pv, X, pc), aty = col_dot(p, L.Acsc, Yp, pc), q = L.qv[pc];
        const double d = (q + px) + aty;
        nrm[1] = cmax(nrm[1], fabs(unscaled ? d / Dg[pc] : d));
        obj[0] += X[pc] * (0.5 * px + q);
    }
    block_max<T>(nrm, L.red);
    block_sum<T>(obj, L.red);
    const double ppri = m == 0 ? 0.0 : nrm[0], pdua = unscaled ? cinv * nrm[1] : nrm[1];
    const double pri0 = p.pri[b], dua0 = p.dua[b];
    const bool take = (ppri < pri0 && pdua < dua0) || (ppri < pri0 && dua0 < 1e-10) || (pdua < dua0 && pri0 < 1e-10);
    if (take) {
        for (int pc = tid; pc < npad; pc += T) {
            const int j = p.pad_var[pc];
            if (j >= 0 && xo) xo[b * n + j] = p.scaling ? Dg[pc] * X[pc] : X[pc];
            p.x[b * npad + pc] = X[pc];
        }
        for (int i = tid; i < m; i += T) {
            if (yo) yo[b * m + i] = p.scaling ? (Eg[i] * Yp[i]) * cinv : Yp[i];
            p.y[b * m + i] = Yp[i];
            p.z[b * m + i] = Zp[i];
        }
    }
    if (tid == 0) {
        p.pstat[b] = take ? 1 : -1;
        if (take) {
            p.obj[b] = p.scaling ? obj[0] * cinv : obj[0];
            p.pri[b] = ppri;
            p.dua[b] = pdua;
        }
    }
}

hipError_t launch_polish(const KParams& p, long B, double* xo, double* yo, hipStream_t st) {
    const size_t lds = lds_solve_bytes(p);
    hipError_t e = hipFuncSetAttribute((const void*)k_polish, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_polish, dim3((unsigned)B), dim3(T), lds, st, p, xo, yo);
    return hipGetLastError();
}

// ------------------------------------------------------------ launcher --
size_t lds_solve_bytes(const KParams& p) { return lds_base_bytes(p); }

size_t lds_kernel_bytes(const KParams& p) {
#ifdef MPCQP_EXPERIMENTAL
    if (p.variant == 16) return lds_dense_bytes(p);
#endif
    if (p.variant == 10 || p.variant == 17) return lds_w2_bytes(p);
#ifdef MPCQP_EXPERIMENTAL
    if (p.variant == 19) return heavy_lds(p);
#endif
    return (p.variant >= 11 && p.variant <= 15) ? lds_solve_bytes_big(p) : lds_solve_bytes(p);
}

template <int NB, int A, int K, int CS, int RS, int W, bool TRI = false>
static hipError_t go(const KParams& p, long B, double* xo, double* yo, int fo, hipStream_t st, size_t lds,
                     KernelRef* ref) {
    auto k = k_solve<NB, A, K, CS, RS, W, TRI>;
    if (ref) { *ref = {(const void*)k, T, lds}; return hipSuccess; }
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3((unsigned)B), dim3(T), lds, st, p, xo, yo, fo);
    return hipGetLastError();
}

// Instantiations: NB = register-resident factor blocks (0: tiles read from the
// workspace), A = coupling rows of F_k, K = gather-list length, CS / RS = columns /
// rows per thread, W = waves per SIMD the register budget is sized for (variants 0, 1, 7
// were sized for 4 and spilled 47 / 161 / 39 VGPRs at the occupancy of 2 they ran at
// anyway; sized for 2 they spill 0 / 19 / 0, round 3), TRI =
// three-phase solve.  variant_fits() is the exact precondition of each.
bool variant_fits(const KParams& p, int v) {
    const int cs = (p.npad + T - 1) / T, rs = (p.m + T - 1) / T;
    if (p.ne && v != 17) return false;  // eliminated variables: the four-wave kernel only
#ifndef MPCQP_EXPERIMENTAL
    // measured and not taken: one-wave 8 / 9, two-wave two-sided 14,
    // 256-thread twisted 15, dense inverse 16, eight-wave 18, one-instance-per-CU dense 19 -- only
    // in the exp / diagnostic builds (MPCQP_BUILD=exp)
    if (v == 8 || v == 9 || v == 14 || v == 15 || v == 16 || v == 18 || v == 19) return false;
#endif
    switch (v) {
        case 0: case 7: return p.nb == 4 && p.amax <= 8 && p.gk <= 6 && cs <= 1 && rs <= 1;
        case 1: return p.nb == 8 && p.amax <= 8 && p.gk <= 8 && cs <= 1 && rs <= 1;
        case 2: return p.nb == 8 && p.amax <= 16 && p.gk <= 8 && cs <= 1 && rs <= 1;
        case 3: return p.nb == 8 && p.amax <= 16 && p.gk <= 8 && cs <= 1 && rs <= 2;
        case 4: return p.gk <= 8 && cs <= 2 && rs <= 4;
        case 5: return p.gk <= 8 && cs <= 4 && rs <= 4;
        case 6: return p.gk <= 16 && cs <= 8 && rs <= 8;
        // the one-wave kernels' rows i = lane + 64 s, s < RS, must cover exactly the padded rows
        // (solve_mpad): RS = 3 for 128 < m <= 192, RS = 4 for 192 < m <= 256
        case 8: return p.nb == 4 && p.amax <= 8 && p.gk <= 6 && solve_mpad(p.m) == 3 * 64 && lds_solve_bytes(p) < 65536;
        case 9: return p.nb == 4 && p.amax <= 8 && p.gk <= 8 && solve_mpad(p.m) == 4 * 64 && lds_solve_bytes(p) < 65536;
        case 10:  // two workgroups per CU (one wave per SIMD): up to 80 KB of LDS each
            return p.nb == 4 && p.amax <= 8 && p.gk <= 6 && p.pk <= 4 && p.m <= 2 * 128 && lds_w2_bytes(p) <= 80 * 1024;
        case 11: case 12: case 13: {
            const int nbm = v == 11 ? 12 : v == 12 ? 18 : 24, csm = v == 11 ? 1 : 2, rsm = v == 13 ? 3 : 2;
            const int csb = (p.npad + kThreadsBig - 1) / kThreadsBig, rsb = (p.m + kThreadsBig - 1) / kThreadsBig;
            return p.nb > 4 && p.nb <= nbm && p.amax <= 16 && p.bmax <= 16 && p.gk <= 8 && csb <= csm && rsb <= rsm &&
                   lds_solve_bytes_big(p) <= 160 * 1024;
        }
        case 15: {  // 256 threads, one wave per SIMD (twisted_solve4): nb <= 18
            const int csb = (p.npad + 255) / 256, rsb = (p.m + 255) / 256;
            return p.nb > 4 && p.nb <= 18 && p.amax <= 16 && p.bmax <= 16 && p.gk <= 8 && csb <= 3 && rsb <= 4 &&
                   lds_solve_bytes_big(p) <= 160 * 1024;
        }
        case 14:
            return p.nb > 4 && p.nb <= 8 && p.amax <= 16 && p.bmax <= 16 && p.gk <= 8 && p.npad <= 256 &&
                   p.m <= 256 && lds_solve_bytes_big(p) <= 160 * 1024;
        case 17: {  // four waves, two workgroups per CU (two waves per SIMD): up to 80 KB of LDS each
            // with eliminated columns: one per upper-half lane (npad <= 256, the fused setup's one
            // column per thread), at most two A nonzeros each (the rhs list LE), three A values per
            // thread in the fused setup
            KParams q2 = p;
            q2.mode = 2;  // the LDS carve of mode 2 (fits may run before KParams::mode is set)
            // (and column lists of up to 8 entries: the slack layout's u_prev columns have 7)
            const bool el = p.ne > 0;
            return p.nb == 4 && p.amax <= 8 && p.gkr <= 6 && p.gkc <= (el ? 8 : 6) && p.pk <= 4 && p.m <= 256 &&
                   p.npad <= (el ? 256 : 128) && p.nnzA <= (el ? 768 : 512) && p.nnzP <= 256 &&
                   (!el || (p.ecnt <= 2 && p.ne <= 128)) && lds_w2_bytes(q2) <= 80 * 1024;
        }
        case 18: {  // eight waves, one workgroup per CU; the gather lists pack 16-bit LDS addresses
            KParams q2 = p;
            q2.mode = 2;  // the LDS carve of mode 2 (fits may run before KParams::mode is set)
            const long mp = solve_mpad(p.m), packed = 8L * (al2(p.nnzA + 1) + al2(p.nnzP + 1) + 4 * mp + 4L * p.npad);
            return p.nb == 8 && p.amax <= 12 && p.gk <= 8 && p.pk <= 8 && p.m <= 512 && p.npad <= 256 &&
                   packed < 65536 && lds_solve_bytes(q2) <= 160 * 1024;
        }
#ifdef MPCQP_EXPERIMENTAL
        case 19: return heavy_fits(p);  // one 512-thread workgroup per QP (solve_heavy.hip)
        case 16:  // dense inverse: one variable per lane pair of a 256-thread workgroup, packed LDS addresses
            return p.n <= kDenseR && p.npad <= 128 && p.gk <= 6 && p.pk <= 4 && p.m <= 2 * 128 &&
                   lds_dense_bytes(p) < 65536;
#endif
        default: return false;
    }
}

int solve_variant(const KParams& p) {
    static const int order[] = {17, 10, 0, 1, 2, 3, 11, 12, 13, 4, 5, 6};  // 8, 9, 14, 16, 18, 19: MPCQP_VARIANT only
    for (int v : order)
        if (variant_fits(p, v)) return v;
    return -1;
}

int solve_threads(int variant) {
    switch (variant) {
        case 8: case 9: return 64;
        case 10: return 128;
        case 11: case 12: case 13: return kThreadsBig;
        case 14: return 128;
        case 15: return 256;
        case 16: return 256;
        case 17: return 256;
        case 18: return 512;
        case 19: return 512;
        default: return T;
    }
}

int solve_mode(int variant) {  // what factorize stores for the variant (KParams::mode)
    switch (variant) {
        case 0: case 8: case 9: case 10: case 17: case 18: case 19: return 2;
        case 1: case 2: case 3: case 7: case 16: return 1;  // (16: no factor stored; dx aliases rb)
        case 11: case 12: case 13: case 14: case 15: return 3;  // two-sided factor (solve_big.hip)
        default: return 0;
    }
}

static hipError_t launch_solve_only(const KParams& p, long B, double* xo, double* yo, int factor_only,
                                    hipStream_t st, KernelRef* ref = nullptr) {
    const size_t lds = lds_solve_bytes(p);
    switch (p.variant) {
        case 0: return go<4, 8, 6, 1, 1, 2, true>(p, B, xo, yo, factor_only, st, lds, ref);
        case 1: return go<8, 8, 8, 1, 1, 2>(p, B, xo, yo, factor_only, st, lds, ref);
        case 2: return go<8, 16, 8, 1, 1, 2>(p, B, xo, yo, factor_only, st, lds, ref);
        case 3: return go<8, 16, 8, 1, 2, 2>(p, B, xo, yo, factor_only, st, lds, ref);
        case 4: return go<0, 32, 8, 2, 4, 2>(p, B, xo, yo, factor_only, st, lds, ref);
        case 5: return go<0, 32, 8, 4, 4, 2>(p, B, xo, yo, factor_only, st, lds, ref);
        case 6: return go<0, 32, 16, 8, 8, 1>(p, B, xo, yo, factor_only, st, lds, ref);
        case 7: return go<4, 8, 6, 1, 1, 2, false>(p, B, xo, yo, factor_only, st, lds, ref);
        case 8: case 9: case 10: case 17: case 18: return launch_solve_wave(p, B, xo, yo, factor_only, st, ref);
#ifdef MPCQP_EXPERIMENTAL
        case 19: {
            if (!factor_only) return launch_solve_heavy(p, B, xo, yo, 0, st, ref);
            KParams q = p;  // setup()'s convexity factorisation: the four-wave kernel's (the same factor)
            q.variant = 17;
            return launch_solve_wave(q, B, xo, yo, factor_only, st, ref);
        }
#endif
#ifdef MPCQP_EXPERIMENTAL
        case 16: return launch_solve_dense(p, B, xo, yo, factor_only, st, ref);
#endif
        case 11: case 12: case 13: case 14: case 15: return launch_solve_big(p, B, xo, yo, factor_only, st, ref);
        default: return hipErrorInvalidValue;
    }
}

int solve_blocks_per_cu(const KParams& p) {
    KernelRef r{};
    if (launch_solve_only(p, 0, nullptr, nullptr, 0, nullptr, &r) != hipSuccess || !r.fn) return -1;
    if (hipFuncSetAttribute(r.fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)r.lds) != hipSuccess) return -1;
    int nblk = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nblk, r.fn, r.threads, r.lds) != hipSuccess) return -1;
    return nblk;
}

hipError_t launch_solve(const KParams& p, long B, double* xo, double* yo, int factor_only, hipStream_t st) {
    hipError_t e = launch_solve_only(p, B, xo, yo, factor_only, st);
    if (e != hipSuccess || factor_only || !p.polish) return e;
    return launch_polish(p, B, xo, yo, st);
}

}  // namespace mpcqp
