// solve_wave.hip -- the ADMM kernel with ONE 64-lane wavefront per QP instance.
//
// Why a wave and not a workgroup: one ADMM iteration of a cfg-2 QP (SURVEY.md §8,
// n = 104, m = 188) is ~7 kFLOP of dependent phases (rhs gather, block solve, row
// update).  Spread over a 256-thread workgroup (solve.hip) every phase boundary
// is an s_barrier between four waves and the iteration costs ~7,000 cycles, almost
// all of it barrier and LDS round trips.  Inside a single wave the phases are
// ordered by the wave's own instruction stream: the compiler drops s_barrier for a
// 64-thread workgroup (it emits only the LDS waitcnt), so a phase boundary costs one
// LDS round trip, and each wave is an independent QP that the four SIMDs of a CU
// run side by side.
//
// Work decomposition (NB <= 4 blocks of S = 32 variables, amax <= 8 coupling rows):
//   lane = (h, r) = (lane / 32, lane % 32) owns the padded columns
//     pc_e = kb_e * 32 + r,  kb_0 = h, kb_1 = 3 - h   (blocks {0,3} / {1,2}: balanced
//     phase-C work), with x, x_prev, q and its column gather lists in registers;
//   constraint rows i = lane + 64 s (s < RS) with y, z, their row gather lists;
//   the factor, in the three-phase form K^{-1} = L^{-T} D^{-1} L^{-1}
//   (solve_phases.h::factorize, mode 2):
//     SB[e][c] = S_{kb_e}^{-1}[r][c]                        (phase B, 64 doubles)
//     GA[q][e] = G_q[lane / 8][4 (lane % 8) + e]            (phase A, pair q = k(k-1)/2 + j)
//     GC[s][q] = G_{j_s, kb_s}[q][r]                        (phase C, transposed use)
// One iteration:
//   rhs   b = sigma x - q + A'(rho z - y)                   -> rb   (LDS)
//   A     c_k = sum_{j<k} G_kj b_j   (8-lane DPP sums)      -> cor  (LDS)
//   B     t_k = S_k^{-1} (b_k + c_k)                        -> tv   (LDS)
//   C     x~_k = t_k + sum_{j>k} G_jk' t_j                  -> xt   (LDS)
//   rows  z~ = A x~, relaxation, projection, y update, w = rho z - y -> w (LDS)
// Reference semantics as solve.hip (OSQP 0.6 osqp_solve, behind
// vehicle_lateral_mpc_slack_increment.py:248 / Control/MPC/mpc_dynamics.py:396).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "setup_r.h"
#include "solve_phases.h"
#include "wave_util.h"

namespace mpcqp {

[[maybe_unused]] constexpr int TW = 64;

#ifdef MPCQP_EXPERIMENTAL  // the one-wave kernels (variants 8, 9): make exp / MPCQP_BUILD=exp
// S^{-1} rows of the lane's two blocks, SB[e][c] = S_{kb_e}^{-1}[r][c] (128 VGPRs)
struct WaveFactor {
    double SB[2][S];
    __device__ __forceinline__ void load(const double* __restrict__ Sg) {
        const int lane = threadIdx.x, h = lane >> 5, r = lane & 31;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const double* src = Sg + (long)(e ? 3 - h : h) * SS + r * S;
#pragma unroll
            for (int c = 0; c < S; ++c) SB[e][c] = src[c];
        }
    }
};

template <int K, int RS>
__global__ __launch_bounds__(TW, 1) void k_solve_w(KParams p, double* __restrict__ xo, double* __restrict__ yo,
                                                   int factor_only) {
    const int lane = threadIdx.x;
    const int h = lane >> 5, r = lane & 31, rr = lane >> 3, ch = lane & 7;
    const int kb0 = h, kb1 = 3 - h;
    constexpr int NB = 4, NP = NB * (NB - 1) / 2;  // exactly four blocks (solve.hip::variant_fits)
    const long b = instance_of(p);
    const int n = p.n, m = p.m, npad = p.npad, nnzP = p.nnzP, nnzA = p.nnzA;
    SL2 C = carve(p);
    SLds& L = C.L;
    const double* Hg = p.H + b * (long)p.nb * SS;
    const double* Sg = p.Si + b * (long)p.nb * SS;

    if (p.err[b]) {  // invalid data (flagged by setup/update): NaN outputs
        for (int j = lane; j < n; j += TW) if (xo) xo[b * n + j] = __builtin_nan("");
        for (int i = lane; i < m; i += TW) if (yo) yo[b * m + i] = __builtin_nan("");
        if (lane == 0) fail_status(p, b);
        return;
    }

#ifdef MPCQP_PHASE_PROF
    long long tph = 0, t0c = 0, t0w = 0;
    const bool prof = p.prof != nullptr;
    if (prof) { t0w = wall_clock64(); t0c = tph = clock64(); if (lane < 16) L.pacc[lane] = 0; }
#define PH(k) if (prof && lane == 0) { const long long t_ = clock64(); L.pacc[k] += t_ - tph; tph = t_; }
#else
#define PH(k)
#endif

    const double cval = p.scal[b * 4 + 0], cinv = p.scal[b * 4 + 1];
    double rho = p.scal[b * 4 + 2];
    const double sigma = p.sigma, alpha = p.alpha;
    const bool warm = p.warm_start != 0;
    for (int e = lane; e < nnzA; e += TW) L.Acsc[e] = p.Ax[b * nnzA + e];
    if (lane == 0) L.Acsc[nnzA] = 0.0;  // the gather lists' padding slot
    for (int v = lane; v < nnzP; v += TW) L.Pv[v] = p.Px[b * nnzP + v];
    if (lane == 0) L.Pv[nnzP] = 0.0;
    const int mp = solve_mpad(m);
    for (int i = lane; i < mp; i += TW) {  // rows >= m: inert padding (l = u = 0, z = 0)
        const bool in = i < m;
        L.lo[i] = in ? p.l[b * m + i] : 0.0;
        L.up[i] = in ? p.u[b * m + i] : 0.0;
        L.ct[i] = in ? p.ct[b * m + i] : 0;
        C.Z[i] = (in && warm) ? p.z[b * m + i] : 0.0;
    }
    for (int pc = lane; pc < npad; pc += TW) {
        L.qv[pc] = p.q[b * npad + pc];
        C.X[pc] = warm ? p.x[b * npad + pc] : 0.0;
    }
    if (lane < S) L.cor[lane] = 0.0;  // block 0 has no phase-A correction
    if (lane < 16) L.res[lane] = 0.0;
    if (lane < 4) L.flag[lane] = 0;

    int status = MPCQP_UNSOLVED_, rho_updates = 0, iter = 0, info_iter = 0;
    bool can_check = false, need_factor = true;
    PH(5)
    // Runs of ADMM iterations up to the next termination / rho-adaptation point
    // alternate with the out-of-line phases; the run state lives in registers and
    // is re-derived from LDS and the workspace at every run start (nothing but
    // scalars is live across a call).
    for (;;) {
        __syncthreads();
        if (need_factor) {  // start, and after a rho change
            need_factor = false;
            // the factorisation scratch aliases ys (and dY, rb, xt, w): y waits in the
            // workspace's y array (the warm-start input at the first factorisation)
            if (iter > 0)
                for (int i = lane; i < m; i += TW) p.y[b * m + i] = L.ys[i];
            const bool ok = factorize_nl<TW>(p.self, b, rho);
            if (!ok) {
                if (iter == 0) {
                    for (int j = lane; j < n; j += TW) if (xo) xo[b * n + j] = __builtin_nan("");
                    for (int i = lane; i < m; i += TW) if (yo) yo[b * m + i] = __builtin_nan("");
                    if (lane == 0) fail_status(p, b);
                    return;
                }
                status = MPCQP_NON_CVX_;
                can_check = true;  // skip the final check_termination
                break;
            }
            if (factor_only) return;
            __syncthreads();
            const bool have_y = iter > 0 || warm;
            for (int i = lane; i < mp; i += TW) L.ys[i] = (have_y && i < m) ? p.y[b * m + i] : 0.0;
            // G blocks -> LDS, rows padded to 8 with zeros: gl[pair][row < 8][32]
            for (int o = lane; o < NP * 8 * S; o += TW) {
                const int q = o >> 8, t = (o >> 5) & 7;
                L.gl[o] = t < p.amax ? Hg[(long)q * p.amax * S + (o & 255)] : 0.0;
            }
            PH(0)
        }
        // ---- run state ----
        WaveFactor RF;
        RF.load(Sg);
        int pcs[2];
        bool cv[2];
        double X[2], Q[2], DX[2];
        // LDS byte addresses of the gathered arrays
        const unsigned abase = lds_addr(L.Acsc), wbase = lds_addr(L.w), xbase = lds_addr(L.xt);
        GatherW<K> cg[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int pc = (e ? kb1 : kb0) * S + r;  // < npad = 4 S
            pcs[e] = pc;
            cv[e] = p.pad_var[pc] >= 0;
            X[e] = C.X[pc];
            Q[e] = L.qv[pc];
            DX[e] = 0.0;
            cg[e].load(p.gcol + pc, npad, abase, wbase);
        }
        GatherW<K> rg[RS];
        double y[RS], Z[RS], dy[RS], rv[RS], rvi[RS];
        const double r_hi = RHO_EQ_OVER_RHO_INEQ * rho;
#pragma unroll
        for (int s = 0; s < RS; ++s) {
            const int i = lane + s * TW;  // < mp
            dy[s] = 0.0;
            if (i < m) rg[s].load(p.grow + i, m, abase, xbase);
            else rg[s].clear(abase + 8u * nnzA, xbase);
            y[s] = L.ys[i];
            Z[s] = C.Z[i];
            const signed char cl = L.ct[i];  // OSQP rho_vec / rho_inv_vec of the row
            rv[s] = cl < 0 ? RHO_MIN : (cl > 0 ? r_hi : rho);
            rvi[s] = cl < 0 ? 1.0 / RHO_MIN : (cl > 0 ? 1.0 / r_hi : 1.0 / rho);
            L.w[i] = rv[s] * Z[s] - y[s];  // w = rho z_prev - y (rho may be new)
        }
        int stop_at = p.max_iter;
        if (p.check_term) stop_at = min(stop_at, (iter / p.check_term + 1) * p.check_term);
        if (p.adaptive_rho && p.rho_interval) stop_at = min(stop_at, (iter / p.rho_interval + 1) * p.rho_interval);
        __syncthreads();
        PH(5)
        while (iter < stop_at) {
            ++iter;
            int opq = 0;
            asm volatile("" : "+s"(opq));  // keeps per-lane LDS addresses out of the register budget
            double* const rb = L.rb + opq;
            double* const cor = L.cor + opq;
            double* const tv = L.tv + opq;
            double* const xt = L.xt + opq;
            // rhs = sigma x_prev - q + A' (rho z_prev - y)
            {
                double av[2][K], wv[2][K];
#pragma unroll
                for (int e = 0; e < 2; ++e)
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        av[e][k] = lds_at(cg[e].e[k] & 0xFFFFu);
                        wv[e][k] = lds_at(cg[e].e[k] >> 16);
                    }
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    double v = sigma * X[e] - Q[e];
#pragma unroll
                    for (int k = 0; k < K; ++k) v += av[e][k] * wv[e][k];
                    rb[pcs[e]] = cv[e] ? v : 0.0;
                }
            }
            __syncthreads();
            PH(1)
            // A: c_k = sum_{j<k} G_kj b_j on rows < 8: lane (rr, ch) takes columns
            // [4 ch, 4 ch + 4) of every pair, 8-lane DPP sums over ch (every lane of
            // the group holds the sum and writes it)
            {
                const double* gq = L.gl + opq + rr * S + 4 * ch;
                double bj[NB - 1][4], ga[NP][4];
#pragma unroll
                for (int j = 0; j < NB - 1; ++j)
#pragma unroll
                    for (int e = 0; e < 4; ++e) bj[j][e] = rb[j * S + 4 * ch + e];
#pragma unroll
                for (int q = 0; q < NP; ++q)
#pragma unroll
                    for (int e = 0; e < 4; ++e) ga[q][e] = gq[q * 8 * S + e];
#pragma unroll
                for (int k = 1; k < NB; ++k) {
                    double acc = 0.0;
#pragma unroll
                    for (int j = 0; j < k; ++j)
#pragma unroll
                        for (int e = 0; e < 4; ++e) acc += ga[k * (k - 1) / 2 + j][e] * bj[j][e];
                    cor[k * S + rr] = reduce8(acc);
                }
            }
            __syncthreads();
            // B: t_kb = S_kb^{-1} (b_kb + c_kb), one full row per lane and block
            double t[2];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int kb = e ? kb1 : kb0;
                const double* bv = rb + kb * S;
                const double* cb = cor + kb * S;
                double v[S], cc[8];
#pragma unroll
                for (int c = 0; c < S; ++c) v[c] = bv[c];
#pragma unroll
                for (int c = 0; c < 8; ++c) cc[c] = cb[c];
#pragma unroll
                for (int c = 0; c < 8; ++c) v[c] += cc[c];
                double a[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int c = 0; c < S; ++c) a[c & 3] += RF.SB[e][c] * v[c];
                t[e] = (a[0] + a[1]) + (a[2] + a[3]);
            }
            tv[kb0 * S + r] = t[0];
            tv[kb1 * S + r] = t[1];
            __syncthreads();
            // C: x~_kb = t_kb + sum_{j>kb} G_{j,kb}' t_j  (t_j rows < 8); the lane's
            // pairs: h = 0: (1,0) (2,0) (3,0);  h = 1: (2,1) (3,1) (3,2)
            double xn[2];
            {
                double d[3], gv[3][8], tq[3][8];
#pragma unroll
                for (int s = 0; s < 3; ++s) {
                    const int j = s < 2 ? s + 1 + h : 3;
                    const int kb = s < 2 ? h : 2 * h;
                    const double* tj = tv + j * S;
                    const double* gc = L.gl + opq + (j * (j - 1) / 2 + kb) * 8 * S + r;
#pragma unroll
                    for (int q = 0; q < 8; ++q) { gv[s][q] = gc[q * S]; tq[s][q] = tj[q]; }
                }
#pragma unroll
                for (int s = 0; s < 3; ++s) {
                    double a0 = 0.0, a1 = 0.0;
#pragma unroll
                    for (int q = 0; q < 8; q += 2) {
                        a0 += gv[s][q] * tq[s][q];
                        a1 += gv[s][q + 1] * tq[s][q + 1];
                    }
                    d[s] = a0 + a1;
                }
                xn[0] = t[0] + (d[0] + d[1]) + (h ? 0.0 : d[2]);
                xn[1] = t[1] + (h ? d[2] : 0.0);
            }
            xt[kb0 * S + r] = xn[0];
            xt[kb1 * S + r] = xn[1];
            // x update (own columns, registers)
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const double xnew = alpha * xn[e] + (1.0 - alpha) * X[e];
                DX[e] = xnew - X[e];
                X[e] = xnew;
            }
            __syncthreads();
            PH(2)
            // z~ = A x~ ; relaxed + projected z ; y ; next w   (padded rows stay 0)
            double zts[RS];
            {
                double av[RS][K], xv[RS][K];
#pragma unroll
                for (int s = 0; s < RS; ++s)
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        av[s][k] = lds_at(rg[s].e[k] & 0xFFFFu);
                        xv[s][k] = lds_at(rg[s].e[k] >> 16);
                    }
#pragma unroll
                for (int s = 0; s < RS; ++s) {
                    double v = av[s][0] * xv[s][0];
#pragma unroll
                    for (int k = 1; k < K; ++k) v += av[s][k] * xv[s][k];
                    zts[s] = v;
                }
            }
#pragma unroll
            for (int s = 0; s < RS; ++s) {
                const int i = lane + opq + s * TW;
                const double zt = zts[s];
                const double zr = alpha * zt + (1.0 - alpha) * Z[s];
                const double zn = __builtin_fmin(__builtin_fmax(zr + rvi[s] * y[s], L.lo[i]), L.up[i]);
                const double dd = rv[s] * (zr - zn);
                Z[s] = zn;
                dy[s] = dd;
                y[s] += dd;
                L.w[i] = rv[s] * zn - y[s];
            }
            __syncthreads();
            PH(3)
        }
        // run state back to LDS for the out-of-line phases
#pragma unroll
        for (int e = 0; e < 2; ++e) { C.X[pcs[e]] = X[e]; L.dx[pcs[e]] = DX[e]; }
#pragma unroll
        for (int s = 0; s < RS; ++s) {
            const int i = lane + s * TW;
            L.ys[i] = y[s]; C.Z[i] = Z[s]; C.dY[i] = dy[s];
        }
        __syncthreads();
        // ---- out-of-line phases (only scalars live across these calls) ----
        can_check = p.check_term && (iter % p.check_term == 0);
        const bool do_rho = p.adaptive_rho && p.rho_interval && (iter % p.rho_interval == 0);
        if (!can_check && !do_rho) break;  // max_iter reached
        update_info_nl<TW>(p.self, b, cinv);
        info_iter = iter;
        bool stop = false;
        if (can_check) {
            status = check_termination_nl<TW>(p.self, b, cval, cinv, 0);
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
        update_info_nl<TW>(p.self, b, cinv);
        info_iter = iter;
        status = check_termination_nl<TW>(p.self, b, cval, cinv, 0);
    }
    const bool has_sol = !(status == MPCQP_PRIMAL_INFEASIBLE_ || status == MPCQP_PRIMAL_INFEASIBLE_INACCURATE_ ||
                           status == MPCQP_DUAL_INFEASIBLE_ || status == MPCQP_DUAL_INFEASIBLE_INACCURATE_ ||
                           status == MPCQP_NON_CVX_);
    if (has_sol) objective_nl<TW>(p.self, cinv);
    if (status == MPCQP_UNSOLVED_) {
        status = check_termination_nl<TW>(p.self, b, cval, cinv, 1);
        if (status == MPCQP_UNSOLVED_) status = MPCQP_MAX_ITER_REACHED_;
    }
    finalize_nl<TW>(p.self, b, xo, yo, cinv, rho, status, info_iter, rho_updates, p.ostat, p.oiter);
#ifdef MPCQP_PHASE_PROF
    if (prof) {
        __syncthreads();
        PH(5)
        if (lane == 0) {
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

#endif  // MPCQP_EXPERIMENTAL

// ---------------------------------------------------------------------------
// Two-wave variant: one 128-thread workgroup (2 waves, on 2 SIMDs) per QP.
// Wave w owns blocks {0, 3} (w = 0) or {1, 2} (w = 1), one block row per lane
// (lane = (h, r): block kb = w ? 1 + h : 3 h, row r), so each wave issues half the
// work of the one-wave kernel with half its registers.  The waves meet at three
// workgroup barriers per iteration (after rhs, after x~, after the row update);
// the cross-block terms of the solve that a wave needs from the other wave's
// blocks (c_k of phase A, and the rows < 8 of t_j that phase C reads) are
// recomputed inside the wave instead of exchanged: phase A is done by both
// waves, and wave 0 recomputes t_1, t_2 (rows < 8), wave 1 recomputes t_3.
// Per-wave LDS for those: cw[w][block][8] (in cor), tw[w][block][8] (in tv).
constexpr int T2 = 128;

template <int K, int RS, int KPK, int K1>
__device__ __forceinline__ void solve_w2_body(const KParams& p, double* __restrict__ xo, double* __restrict__ yo,
                                              int factor_only) {
    static_assert(RS == 2, "rows i = tid and tid + 128");
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int h = lane >> 5, r = lane & 31, rr = lane >> 3, ch = lane & 7;
    const int kb = w ? 1 + h : 3 * h;          // own block
    const int jr = w ? 3 : 1 + h;              // block of the recomputed t rows
    const int rq = r >> 2, cq = r & 3;         // recomputed row / column chunk
    constexpr int NB = 4, NP = NB * (NB - 1) / 2;  // exactly four blocks (solve.hip::variant_fits)
    const long b = instance_of(p);
    const int n = p.n, m = p.m, npad = p.npad, nnzP = p.nnzP, nnzA = p.nnzA;
    SL2 C = carve(p);
    SLds& L = C.L;
    const double* Hg = p.H + b * (long)p.nb * SS;
    // S_k^{-1} stays in LDS after the carve (lds_w2_bytes): at one wave per SIMD two
    // workgroups share a CU, so the LDS is there; nothing goes to / comes from the workspace
    double* const Sg = C.L.Acsc + 2 * ((lds_base_bytes(p) + 15) / 16);

    if (p.err[b]) {  // invalid data (flagged by setup/update): NaN outputs
        for (int j = tid; j < n; j += T2) if (xo) xo[b * n + j] = __builtin_nan("");
        for (int i = tid; i < m; i += T2) if (yo) yo[b * m + i] = __builtin_nan("");
        if (tid == 0) fail_status(p, b);
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
#ifdef MPCQP_CHECK_PROF  // diagnostic: slots 12-14 time the run end / reductions / certificates of a check
#define PHL(k) PH(2)
#define PHC(k) PH(k)
#else
#define PHL(k) PH(k)
#define PHC(k)
#endif

    const double cval = p.scal[b * 4 + 0], cinv = p.scal[b * 4 + 1];
    double rho = p.scal[b * 4 + 2];
    const double sigma = p.sigma, alpha = p.alpha;
    const bool warm = p.warm_start != 0;
    for (int e = tid; e < nnzA; e += T2) L.Acsc[e] = p.Ax[b * nnzA + e];
    if (tid == 0) L.Acsc[nnzA] = 0.0;  // the gather lists' padding slot
    for (int v = tid; v < nnzP; v += T2) L.Pv[v] = p.Px[b * nnzP + v];
    if (tid == 0) L.Pv[nnzP] = 0.0;
    const int mp = solve_mpad(m);
    for (int i = tid; i < mp; i += T2) {  // rows >= m: inert padding (l = u = 0, z = 0)
        const bool in = i < m;
        L.lo[i] = in ? p.l[b * m + i] : 0.0;
        L.up[i] = in ? p.u[b * m + i] : 0.0;
        L.ct[i] = in ? p.ct[b * m + i] : 0;
        C.Z[i] = (in && warm) ? p.z[b * m + i] : 0.0;
    }
    for (int pc = tid; pc < npad; pc += T2) {
        L.qv[pc] = p.q[b * npad + pc];
        C.X[pc] = warm ? p.x[b * npad + pc] : 0.0;
    }
    if (tid < 16) L.cor[(tid >> 3) * 32 + (tid & 7)] = 0.0;  // cw[w][0][*]: block 0 has no correction
    if (tid < 16) L.res[tid] = 0.0;
    if (tid < 4) L.flag[tid] = 0;

    int status = MPCQP_UNSOLVED_, rho_updates = 0, iter = 0, info_iter = 0;
    bool can_check = false, need_factor = true;
    // Loop-invariant per-lane data from global memory (the plan's gather lists, the
    // scalings D and E): loaded after each factorisation (which is a call: nothing
    // vector-valued is live across it), kept in registers across the runs and the
    // inline termination checks in between.
    const int pc = kb * S + r;
    const unsigned abase = lds_addr(L.Acsc), wbase = lds_addr(L.w), xbase = lds_addr(L.xt);
    const unsigned Xbase = lds_addr(C.X);
    bool cv = false;
    double Dv = 1.0, Ev[RS];
    // row gather lists: slot 0 (rows < 128) K entries, slot 1 (rows >= 128) K1 <= K --
    // the plan's row order often puts the short rows last (cfg 2: the box rows, one
    // nonzero each, are rows 84..187), so slot 1 skips the zero-padded entries
    GatherW<K> cg, rg0;
    GatherW<K1> rg1;
    GatherW<KPK> pg;  // the column's P list (addresses of Pv / X), for the inline check
    PH(5)
    for (;;) {
        __syncthreads();
        if (need_factor) {  // start, and after a rho change
            need_factor = false;
            // the factorisation scratch aliases ys: y waits in the workspace's y array
            if (iter > 0) {
                for (int i = tid; i < m; i += T2) p.y[b * m + i] = L.ys[i];
                __syncthreads();  // every ys read is done before factorize_w2's scratch overwrites it
            }
            const bool ok = factorize_nl<T2>(p.self, b, rho, Sg);
            if (!ok) {
                if (iter == 0) {
                    for (int j = tid; j < n; j += T2) if (xo) xo[b * n + j] = __builtin_nan("");
                    for (int i = tid; i < m; i += T2) if (yo) yo[b * m + i] = __builtin_nan("");
                    if (tid == 0) fail_status(p, b);
                    return;
                }
                status = MPCQP_NON_CVX_;
                can_check = true;  // skip the final check_termination
                break;
            }
            if (factor_only) return;
            __syncthreads();
            const bool have_y = iter > 0 || warm;
            for (int i = tid; i < mp; i += T2) L.ys[i] = (have_y && i < m) ? p.y[b * m + i] : 0.0;
            // G blocks -> LDS, rows padded to 8 with zeros, plus one all-zero pair (index NP):
            // gl[pair][row < 8][32]
            for (int o = tid; o < (NP + 1) * 8 * S; o += T2) {
                const int q = o >> 8, t = (o >> 5) & 7;
                L.gl[o] = (q < NP && t < p.amax) ? Hg[(long)q * p.amax * S + (o & 255)] : 0.0;
            }
            cv = p.pad_var[pc] >= 0;
            cg.load(p.gcol + pc, npad, abase, wbase);
            pg.load(p.gpsym + pc, npad, lds_addr(L.Pv), Xbase);
            Dv = p.D[b * npad + pc];
#pragma unroll
            for (int s = 0; s < RS; ++s) {
                const int i = min(tid + s * T2, mp - 1);
                Ev[s] = i < m ? p.E[b * m + i] : 1.0;
            }
            {
                const int i0 = tid, i1 = min(tid + T2, mp - 1);
                if (i0 < m) rg0.load(p.grow + i0, m, abase, xbase);
                else rg0.clear(abase + 8u * nnzA, xbase);
                if (i1 < m) rg1.load(p.grow + i1, m, abase, xbase);
                else rg1.clear(abase + 8u * nnzA, xbase);
            }
            PH(0)
        }
        // ---- run state ----
        double SB[S], SR[8];
        {
            const double* src = Sg + (long)kb * SS + r * S;
#pragma unroll
            for (int c = 0; c < S; c += 2) ld2(src + c, SB[c], SB[c + 1]);
            const double* srr = Sg + (long)jr * SS + rq * S + 8 * cq;
#pragma unroll
            for (int i = 0; i < 8; i += 2) ld2(srr + i, SR[i], SR[i + 1]);
        }
        double X = C.X[pc], DX = 0.0;
        const double Q = L.qv[pc];
        // phase-C slots (pair, j) of the lane; pair NP is the zero block.  Block 0 needs
        // three pairs and block 3 none, so wave 0's upper half (block 3's rows) takes block
        // 0's pair (3,0) and hands its partial sum over with a half-wave swap: two slots
        // per lane in both waves.
        int gslot[2], tslot[2];
        {
            int pr[2], jj[2];
            if (w == 0 && h == 0) { pr[0] = 0; jj[0] = 1; pr[1] = 1; jj[1] = 2; }
            else if (w == 0)      { pr[0] = 3; jj[0] = 3; pr[1] = NP; jj[1] = 3; }
            else if (h == 0)      { pr[0] = 2; jj[0] = 2; pr[1] = 4; jj[1] = 3; }
            else                  { pr[0] = 5; jj[0] = 3; pr[1] = NP; jj[1] = 3; }
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                gslot[s] = lds_addr(L.gl + pr[s] * 8 * S + r);
                tslot[s] = lds_addr(L.tv + w * 32 + jj[s] * 8);
            }
        }
        double y[RS], Z[RS], dy[RS], rv[RS], rvi[RS];
        int ri[RS];
        const double r_hi = RHO_EQ_OVER_RHO_INEQ * rho;
#pragma unroll
        for (int s = 0; s < RS; ++s) {
            const int i = min(tid + s * T2, mp - 1);  // lanes past the padded rows repeat the inert last row
            ri[s] = i;
            dy[s] = 0.0;
            y[s] = L.ys[i];
            Z[s] = C.Z[i];
            const signed char cl = L.ct[i];  // OSQP rho_vec / rho_inv_vec of the row
            rv[s] = cl < 0 ? RHO_MIN : (cl > 0 ? r_hi : rho);
            rvi[s] = cl < 0 ? 1.0 / RHO_MIN : (cl > 0 ? 1.0 / r_hi : 1.0 / rho);
        }
        __syncthreads();  // every ys / Z read before w is written
#pragma unroll
        for (int s = 0; s < RS; ++s) L.w[ri[s]] = rv[s] * Z[s] - y[s];  // w = rho z_prev - y (rho may be new)
        int stop_at = p.max_iter;
        if (p.check_term) stop_at = min(stop_at, (iter / p.check_term + 1) * p.check_term);
        if (p.adaptive_rho && p.rho_interval) stop_at = min(stop_at, (iter / p.rho_interval + 1) * p.rho_interval);
        __syncthreads();
        PH(5)
        double* const cw = L.cor + w * 32;  // this wave's c_k rows < 8
        double* const tw = L.tv + w * 32;   // this wave's t_j rows < 8
        while (iter < stop_at) {
            ++iter;
            // rhs = sigma x_prev - q + A' (rho z_prev - y), own column
            {
                double av[K], wv[K];
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    av[k] = lds_at(cg.e[k] & 0xFFFFu);
                    wv[k] = lds_at(cg.e[k] >> 16);
                }
                double v = sigma * X - Q;
#pragma unroll
                for (int k = 0; k < K; ++k) v += av[k] * wv[k];
                L.rb[pc] = cv ? v : 0.0;
            }
            __syncthreads();
            PH(1)
            // A (both waves): c_k = sum_{j<k} G_kj b_j, rows < 8
            {
                const double* gq = L.gl + rr * S + 4 * ch;
                double bj[NB - 1][4], ga[NP][4];
#pragma unroll
                for (int j = 0; j < NB - 1; ++j)
#pragma unroll
                    for (int e = 0; e < 4; e += 2) ld2(L.rb + j * S + 4 * ch + e, bj[j][e], bj[j][e + 1]);
#pragma unroll
                for (int q = 0; q < NP; ++q)
#pragma unroll
                    for (int e = 0; e < 4; e += 2) ld2(gq + q * 8 * S + e, ga[q][e], ga[q][e + 1]);
#pragma unroll
                for (int k = 1; k < NB; ++k) {
                    double acc = 0.0;
#pragma unroll
                    for (int j = 0; j < k; ++j)
#pragma unroll
                        for (int e = 0; e < 4; ++e) acc += ga[k * (k - 1) / 2 + j][e] * bj[j][e];
                    cw[k * 8 + rr] = reduce8(acc);
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            PHL(12)
            // B: own row t_kb[r] = S_kb^{-1}[r] (b_kb + c_kb); recomputed rows < 8 of t_jr
            double t;
            {
                double v[S], cc[8];
#pragma unroll
                for (int c = 0; c < S; c += 2) ld2(L.rb + kb * S + c, v[c], v[c + 1]);
#pragma unroll
                for (int c = 0; c < 8; c += 2) ld2(cw + kb * 8 + c, cc[c], cc[c + 1]);
                double u[8], uc[8];
#pragma unroll
                for (int i = 0; i < 8; i += 2) {
                    ld2(L.rb + jr * S + 8 * cq + i, u[i], u[i + 1]);
                    ld2(cw + jr * 8 + i, uc[i], uc[i + 1]);
                }
#pragma unroll
                for (int c = 0; c < 8; ++c) v[c] += cc[c];
                double a[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int c = 0; c < S; ++c) a[c & 3] += SB[c] * v[c];
                t = (a[0] + a[1]) + (a[2] + a[3]);
                double a0 = 0.0, a1 = 0.0;
#pragma unroll
                for (int i = 0; i < 8; i += 2) {
                    a0 += SR[i] * (cq == 0 ? u[i] + uc[i] : u[i]);
                    a1 += SR[i + 1] * (cq == 0 ? u[i + 1] + uc[i + 1] : u[i + 1]);
                }
                double tr = a0 + a1;
                tr += dpp<0xB1>(tr);
                tr += dpp<0x4E>(tr);  // sum over the quad (the four column chunks)
                tw[jr * 8 + rq] = tr;
                if (r < 8) tw[kb * 8 + r] = t;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            PHL(13)
            // C: x~_kb[r] = t + sum_s G_{pair_s}[q][r] t_{j_s}[q]
            {
                double gv[2][8], tq[2][8];
#pragma unroll
                for (int s = 0; s < 2; ++s) {
#pragma unroll
                    for (int q = 0; q < 8; ++q) gv[s][q] = lds_at(gslot[s] + q * S * 8);
#pragma unroll
                    for (int q = 0; q < 8; q += 2) {
                        lds_at2(tslot[s] + q * 8, tq[s][q], tq[s][q + 1]);
                    }
                }
                double a0 = 0.0, a1 = 0.0;
#pragma unroll
                for (int s = 0; s < 2; ++s)
#pragma unroll
                    for (int q = 0; q < 8; q += 2) {
                        a0 += gv[s][q] * tq[s][q];
                        a1 += gv[s][q + 1] * tq[s][q + 1];
                    }
                double d = a0 + a1;
                if (w == 0) {  // block 0 (lower half) + its pair (3,0) from the upper half; block 3: t
                    const unsigned lo = (unsigned)__double2loint(d), hi = (unsigned)__double2hiint(d);
                    const auto l2 = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
                    const auto h2 = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
                    const double dl0 = __hiloint2double((int)h2[0], (int)l2[0]);  // lower half's partial
                    const double dl1 = __hiloint2double((int)h2[1], (int)l2[1]);  // upper half's partial
                    d = h ? 0.0 : dl0 + dl1;
                }
                const double xn = t + d;
                L.xt[pc] = xn;
                const double xnew = alpha * xn + (1.0 - alpha) * X;
                DX = xnew - X;
                X = xnew;
            }
            __syncthreads();
            PHL(14)
            // z~ = A x~ ; relaxed + projected z ; y ; next w
            {
                double av0[K], xv0[K], av1[K1], xv1[K1], lo[RS], up[RS], zts[RS];
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    av0[k] = lds_at(rg0.e[k] & 0xFFFFu);
                    xv0[k] = lds_at(rg0.e[k] >> 16);
                }
#pragma unroll
                for (int k = 0; k < K1; ++k) {
                    av1[k] = lds_at(rg1.e[k] & 0xFFFFu);
                    xv1[k] = lds_at(rg1.e[k] >> 16);
                }
#pragma unroll
                for (int s = 0; s < RS; ++s) {
                    lo[s] = L.lo[ri[s]];
                    up[s] = L.up[ri[s]];
                }
                zts[0] = av0[0] * xv0[0];
#pragma unroll
                for (int k = 1; k < K; ++k) zts[0] += av0[k] * xv0[k];
                zts[1] = av1[0] * xv1[0];
#pragma unroll
                for (int k = 1; k < K1; ++k) zts[1] += av1[k] * xv1[k];
#pragma unroll
                for (int s = 0; s < RS; ++s) {
                    const double zt = zts[s];
                    const double zr = alpha * zt + (1.0 - alpha) * Z[s];
                    const double zn = __builtin_fmin(__builtin_fmax(zr + rvi[s] * y[s], lo[s]), up[s]);
                    const double dd = rv[s] * (zr - zn);
                    Z[s] = zn;
                    dy[s] = dd;
                    y[s] += dd;
                    L.w[ri[s]] = rv[s] * zn - y[s];
                }
            }
            __syncthreads();
            PH(3)
        }
        // run state back to LDS for the out-of-line phases
        C.X[pc] = X;
        L.dx[pc] = DX;
#pragma unroll
        for (int s = 0; s < RS; ++s) { L.ys[ri[s]] = y[s]; C.Z[ri[s]] = Z[s]; C.dY[ri[s]] = dy[s]; }
        __syncthreads();
        PHC(12)
        can_check = p.check_term && (iter % p.check_term == 0);
        const bool do_rho = p.adaptive_rho && p.rho_interval && (iter % p.rho_interval == 0);
        if (!can_check && !do_rho) break;  // max_iter reached
        info_iter = iter;
        bool stop = false;
        {
            // ---- inline update_info + check_termination (OSQP 0.6 update_info,
            // check_termination, is_primal_infeasible, is_dual_infeasible; the same
            // arithmetic as solve_phases.h::update_info_ph / check_termination_ph) on the
            // register-resident gather lists: no dependent global loads, no calls ----
            const bool unscale = p.scaling && !p.scaled_term;
            const unsigned ysbase = lds_addr(L.ys), dYbase = lds_addr(C.dY), dxbase = lds_addr(L.dx);
            double mx[17], sm[2] = {0.0, 0.0}, adx[RS];
#pragma unroll
            for (int k = 0; k < 17; ++k) mx[k] = 0.0;
#pragma unroll
            for (int s = 0; s < RS; ++s) {  // rows: A x, z, the projected delta y, A dx
                const bool ok = tid + s * T2 < m;
                double ax = 0.0, ad = 0.0;
                auto rowdots = [&](const auto& g) __attribute__((always_inline)) {
                    constexpr int KK = std::extent_v<std::remove_reference_t<decltype(g.e)>>;
#pragma unroll
                    for (int k = 0; k < KK; ++k) {
                        const unsigned e = g.e[k], va = e >> 16;
                        const double a = lds_at(e & 0xFFFFu);
                        ax += a * lds_at(va - xbase + Xbase);
                        ad += a * lds_at(va - xbase + dxbase);
                    }
                };
                if (s == 0) rowdots(rg0);
                else rowdots(rg1);
                adx[s] = ad;
                const double zi = Z[s], pr = ax - zi, ei = 1.0 / Ev[s];
                const double lo = L.lo[ri[s]], up = L.up[ri[s]];
                double d = dy[s];
                if (up > OSQP_INFTY * MIN_SCALING) d = (lo < -OSQP_INFTY * MIN_SCALING) ? 0.0 : cmin(d, 0.0);
                else if (lo < -OSQP_INFTY * MIN_SCALING) d = cmax(d, 0.0);
                if (ok) {
                    mx[0] = vmax(mx[0], fabs(ei * pr));
                    mx[2] = vmax(mx[2], fabs(ei * zi));
                    mx[3] = vmax(mx[3], fabs(ei * ax));
                    mx[7] = vmax(mx[7], fabs(pr));
                    mx[9] = vmax(mx[9], fabs(zi));
                    mx[10] = vmax(mx[10], fabs(ax));
                    mx[14] = vmax(mx[14], fabs(unscale ? Ev[s] * d : d));
                    sm[0] += up * cmax(d, 0.0) + lo * cmin(d, 0.0);
                    C.dY[ri[s]] = d;  // projected in place, as OSQP's is_primal_infeasible
                }
            }
            {  // the lane's column: P x, A' y, P dx, and the delta x norm
                double px = 0.0, pdx = 0.0, aty = 0.0;
#pragma unroll
                for (int k = 0; k < KPK; ++k) {
                    const unsigned e = pg.e[k], va = e >> 16;
                    const double pv = lds_at(e & 0xFFFFu);
                    px += pv * lds_at(va);
                    pdx += pv * lds_at(va - Xbase + dxbase);
                }
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const unsigned e = cg.e[k];
                    aty += lds_at(e & 0xFFFFu) * lds_at((e >> 16) - wbase + ysbase);
                }
                if (cv) {
                    const double d = (Q + px) + aty, di = 1.0 / Dv;
                    mx[1] = fabs(di * d);
                    mx[4] = fabs(di * Q);
                    mx[5] = fabs(di * aty);
                    mx[6] = fabs(di * px);
                    mx[8] = fabs(d);
                    mx[11] = fabs(Q);
                    mx[12] = fabs(aty);
                    mx[13] = fabs(px);
                    mx[15] = fabs(unscale ? Dv * DX : DX);
                    mx[16] = fabs(unscale ? pdx * di : pdx);
                }
            }
            // q' dx with the out-of-line phases' column-per-thread order (column tid)
            if (p.pad_var[tid] >= 0) sm[1] = L.qv[tid] * L.dx[tid];
            block_max_sum_tr<T2, 17, 2>(mx, sm, L.red);
            PHC(13)
            Res R;
            if (unscale) {
                R.pri = mx[0]; R.dua = cinv * mx[1];
                R.nz = mx[2]; R.nax = mx[3]; R.nq = mx[4]; R.naty = mx[5]; R.npx = mx[6];
            } else {
                R.pri = mx[7]; R.dua = mx[8];
                R.nz = mx[9]; R.nax = mx[10]; R.nq = mx[11]; R.naty = mx[12]; R.npx = mx[13];
            }
            R.rpri = mx[7]; R.rdua = mx[8]; R.rz = mx[9]; R.rax = mx[10]; R.rq = mx[11]; R.raty = mx[12]; R.rpx = mx[13];
            if (m == 0) R.pri = 0.0;
            if (tid == 0) R.save(L.res);
            if (can_check) {
                int st = MPCQP_UNSOLVED_;
                double obj = 0.0;
                bool done = false;
                if (R.pri > OSQP_INFTY || R.dua > OSQP_INFTY) {
                    st = MPCQP_NON_CVX_;
                    obj = __builtin_nan("");
                    done = true;
                } else {
                    const bool prim_ok = m == 0 || R.pri < p.eps_abs + p.eps_rel * cmax(R.nz, R.nax);
                    double mxd = cmax(cmax(R.nq, R.naty), R.npx);
                    if (unscale) mxd *= cinv;
                    const bool dual_ok = R.dua < p.eps_abs + p.eps_rel * mxd;
                    bool prim_inf = false, dual_inf = false;
                    if (!prim_ok || !dual_ok) {  // infeasibility certificates (uniform branches)
                        // OSQP's is_primal_infeasible / is_dual_infeasible evaluate their tests in
                        // order and return at the first that fails: the reduced norms and sums
                        // decide whether the gathered A'dy maximum / the A dx row test is needed
                        const double norm_dy = mx[14], norm_dx = mx[15], epi = p.eps_pinf, edi = p.eps_dinf;
                        const double cs = unscale ? cval : 1.0;
                        if (!prim_ok && m != 0 && norm_dy > epi && sm[0] < epi * norm_dy) {
                            __syncthreads();  // the projected delta y
                            double na[1] = {0.0};
                            double a = 0.0;
#pragma unroll
                            for (int k = 0; k < K; ++k) {
                                const unsigned e = cg.e[k];
                                a += lds_at(e & 0xFFFFu) * lds_at((e >> 16) - wbase + dYbase);
                            }
                            if (cv) na[0] = fabs(unscale ? a * (1.0 / Dv) : a);
                            block_max<T2, 1>(na, L.red);
                            prim_inf = na[0] < epi * norm_dy;
                        }
                        if (!dual_ok && norm_dx > edi && sm[1] < cs * edi * norm_dx && mx[16] < cs * edi * norm_dx) {
                            bool viol = false;
#pragma unroll
                            for (int s = 0; s < RS; ++s) {
                                if (!(tid + s * T2 < m)) continue;
                                const double ar = unscale ? adx[s] * (1.0 / Ev[s]) : adx[s];
                                const double lo = L.lo[ri[s]], up = L.up[ri[s]];
                                if ((up < OSQP_INFTY * MIN_SCALING && ar > edi * norm_dx) ||
                                    (lo > -OSQP_INFTY * MIN_SCALING && ar < -edi * norm_dx))
                                    viol = true;
                            }
                            dual_inf = !block_any<T2>(viol, L.flag);
                        }
                    }
                    if (prim_ok && dual_ok) {
                        st = MPCQP_SOLVED_;
                        done = true;
                    } else if (prim_inf) {
                        st = MPCQP_PRIMAL_INFEASIBLE_;
                        obj = OSQP_INFTY;
                        if (tid == 0) L.flag[3] = unscale;
                        done = true;
                    } else if (dual_inf) {
                        st = MPCQP_DUAL_INFEASIBLE_;
                        obj = -OSQP_INFTY;
                        if (tid == 0) L.flag[2] = unscale;
                        done = true;
                    }
                }
                __syncthreads();
                if (done && tid == 0) { L.flag[1] = st; L.res[14] = obj; }
                __syncthreads();
                status = done ? st : MPCQP_UNSOLVED_;
                stop = done;
            }
        }
        PHC(14)
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
        update_info_nl<T2>(p.self, b, cinv);
        info_iter = iter;
        status = check_termination_nl<T2>(p.self, b, cval, cinv, 0);
    }
    const bool has_sol = !(status == MPCQP_PRIMAL_INFEASIBLE_ || status == MPCQP_PRIMAL_INFEASIBLE_INACCURATE_ ||
                           status == MPCQP_DUAL_INFEASIBLE_ || status == MPCQP_DUAL_INFEASIBLE_INACCURATE_ ||
                           status == MPCQP_NON_CVX_);
    if (has_sol) objective_nl<T2>(p.self, cinv);
    if (status == MPCQP_UNSOLVED_) {
        status = check_termination_nl<T2>(p.self, b, cval, cinv, 1);
        if (status == MPCQP_UNSOLVED_) status = MPCQP_MAX_ITER_REACHED_;
    }
    finalize_nl<T2>(p.self, b, xo, yo, cinv, rho, status, info_iter, rho_updates, p.ostat, p.oiter);
#ifdef MPCQP_PHASE_PROF
    if (prof) {
        __syncthreads();
        PH(5)
        if (tid == 0) {
#pragma unroll
            for (int k = 0; k < 6; ++k) p.prof[b * kProfSlots + k] = L.pacc[k];
#pragma unroll
            for (int k = 8; k < 15; ++k) p.prof[b * kProfSlots + k] = L.pacc[k];
#ifndef MPCQP_CHECK_PROF
            p.prof[b * kProfSlots + 2] = L.pacc[12] + L.pacc[13] + L.pacc[14];
#endif
            p.prof[b * kProfSlots + 6] = clock64() - t0c;
            p.prof[b * kProfSlots + 7] = wall_clock64() - t0w;
            p.prof[b * kProfSlots + 15] = t0w;  // absolute start (100 MHz): dispatch order / residency
        }
    }
#endif
#undef PH
#undef PHL
#undef PHC
}

// the kernel: the solve, then (last workgroup only) the dispatch order of the next launch
template <int K, int RS, int KPK, int K1>
__global__ __launch_bounds__(T2, 1) void k_solve_w2(KParams p, double* __restrict__ xo, double* __restrict__ yo,
                                                    int factor_only) {
    solve_w2_body<K, RS, KPK, K1>(p, xo, yo, factor_only);
    extern __shared__ __attribute__((aligned(16))) double sm[];
    order_epilogue<T2>(p, (int*)sm);
}

// Fused setup + solve (mpcqp_setup_solve_device): the workgroup Ruiz-scales its
// instance with the register-list setup (setup_r.h, the same arithmetic as k_setup /
// k_setup_r), then solves it.  Everything the solve reads from the workspace was
// written by this workgroup before the barrier, so no second kernel, no launch gap and
// no setup kernel in front of the slowest instance.
template <int K, int RS, int KPK, int K1, int SK, int SRS, int SAS, int SPS>
__global__ __launch_bounds__(T2, 1) void k_setup_solve_w2(KParams p, const double* __restrict__ Px_in,
                                                          const double* __restrict__ Ax_in,
                                                          const double* __restrict__ q_in,
                                                          const double* __restrict__ l_in,
                                                          const double* __restrict__ u_in, double* __restrict__ xo,
                                                          double* __restrict__ yo) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    setup_r_body<T2, SK, 4, SRS, SAS, SPS>(p, instance_of(p), Px_in, Ax_in, q_in, l_in, u_in, sm);
    __syncthreads();
    solve_w2_body<K, RS, KPK, K1>(p, xo, yo, 0);
    order_epilogue<T2>(p, (int*)sm);
}

// ---------------------------------------------------------------------------
// Four-wave variant (variant 17, k_solve_w4 / k_setup_solve_w4): one 256-thread
// workgroup per QP, wave k owns block k.  Lane (h, r) keeps row r of S_k^{-1}, columns
// [16 h, 16 h + 16) (32 VGPRs instead of the two-wave kernel's 64 + 16), and row i = tid
// of A.  Per iteration:
//   rhs   column k S + r (both halves compute it, the lower half stores)   -> barrier
//   A     c_k = sum_{j<k} G_kj b_j, rows < 8 (wave k only its own block)  -> wave sync
//   B     t_k[r] = S_k^{-1}[r] (b_k + c_k): half-row sums + permlane32     -> barrier
//   C     x~_k[r] = t_k[r] + sum_{j>k} G_jk' t_j[0, 8): the pairs split over the halves
//   rows  z~ = A x~ (one row per lane), relaxation, projection, y, w      -> barrier
// Four barriers instead of three, but each wave issues about 60 % of a two-wave wave's
// instructions, and the factorisation pre-pivots the four blocks at once
// (solve_phases.h::factorize_w4).  Operands that do not change within a run (the row's
// and half-column's A values, the row bounds, phase A's and phase C's G values) are
// loaded into registers at the run start: fewer LDS reads (and waits) per iteration on
// every wave's path.  MPCQP_VARIANT=17 (A/B against variant 10).
constexpr int T4 = 256;

// EL: the plan has eliminated columns (plan.h Plan::eown; the slack layouts).  The upper
// half-wave lane (1, r) of wave w then owns the eliminated column pe = eown[w S + r] of its
// block column's variable: it folds -ec b_pe into its half of the block column's rhs sum
// (b_p - (K_pj / K_jj) b_j, no extra exchange), keeps x_pe, q_pe and b_pe in its registers,
// and after phase C sets  x~_pe = ed b_pe - ec x~_p  (ed = 1 / K_jj, ec = K_pj / K_jj,
// factorize_w4) -- the elementwise back-substitution of the scalar Schur complement --
// which the rows phase reads from xt like any other column.  Its termination-check column
// is pe (the lower half keeps the block column).
// DK (dense inverse, no eliminated columns): the three-phase solve x~ = L' D L b (L = I + the
// G blocks below the diagonal, D = diag(S_k^{-1}); phases A, B, C above) replaced by one
// product with M^{-1} = L' D L formed explicitly after each factorisation.  Lane (h, r) of
// wave a keeps row a S + r of M^{-1} over the real columns of blocks 2 h and 2 h + 1 (the
// first NBC of each: plan.cpp's balanced merge keeps every block at <= NBC real columns):
//   rhs   -> barrier ->   x~ = M^{-1} b: 2 NBC FMAs per lane, one permlane32   -> barrier -> rows
// Three barriers a step instead of four, and no phase whose length depends on the block
// (the three-phase form's wave 3 runs three phase-A pairs, wave 0 two phase-C slots).
// Block (a, b) of L' D L is  sum over k >= max(a, b) of  L_ka' S_k^{-1} L_kb  (L_kk = I, L_kj
// = G_kj for j < k, nonzero rows < QR):
//   [a = b] S_a^{-1}[i][c]
//   + sum_q S_a^{-1}[i][q] G_ab[q][c]                       (a > b)
//   + sum_q G_ba[q][i] S_b^{-1}[q][c]                       (b > a)
//   + sum_{k > a, k > b} sum_q V_ka[i][q] G_kb[q][c],  V_ka[i][q] = sum_p G_ka[p][i] S_k^{-1}[p][q]
// Each term is a sum of rank-one row updates: a lane coefficient times a row read from LDS
// by broadcast (one row per half-wave).  G blocks come from the LDS copy gl (pair (k, j) at
// k (k - 1) / 2 + j, pair NP the zero block: a lane whose b does not satisfy the term's
// condition reads zeros), S_k^{-1} from the LDS tiles Sg.
// M^{-1} = L' D L into the instance's Kd rows, in 4 x 8 tiles: wave a forms block row a,
// lanes [16 b, 16 b + 16) block (a, b), lane l16 = lane & 15 the rows 4 (l16 >> 1) .. + 3 and
// columns 16 (l16 & 1) .. + 15 in two passes of 8 -- an outer-product update per term step
// (4 coefficients, 8 row values, 32 FMAs) instead of a 28-wide row per lane (28 values for 28
// FMAs): 3/8 of the LDS reads per FMA, the wave's steps 5 [a > 0] + 5 [a < 3] + 5 (3 - a) (pair NP, the
// zero block, for the blocks a term does not apply to).  Element (i, c) of block (a, b) goes
// to the dense-row slot of its lane (a, b & 1, i): pair j / 2 of the lane's row, j = c (b < 2)
// or NB0 + c (b >= 2), c below NB0 / NB1 only.  Stored through global memory, read back by
// other lanes after the next workgroup barrier.
template <int QR, int NB0, int NB1>
__device__ __forceinline__ void form_dense_rows(__attribute__((address_space(1))) dpair* kd, const double* Sg,
                                                const double* gl, int a, int lane) {
    constexpr int NP = 6, T4_ = 256, TC = 8;  // TC: tile columns per pass (two passes of the lane's 16)
    auto pidx = [](int x, int y) { return y < x ? x * (x - 1) / 2 + y : NP; };
    const int bq = lane >> 4, l16 = lane & 15, i0 = 4 * (l16 >> 1);
    const double* const Ta = Sg + a * SS;
    const int nbs = (bq >> 1) ? NB1 : NB0, jb = (bq >> 1) ? NB0 : 0;
    const unsigned t0 = (unsigned)(a * 64 + (bq & 1) * 32 + i0);
#pragma unroll 1
    for (int pass = 0; pass < 2; ++pass) {
        const int c0 = 16 * (l16 & 1) + TC * pass;
        double acc[4][TC];
        {   // [a = b] the tile of S_a^{-1}
            const double* src = Sg + bq * SS + i0 * S + c0;
            const bool diag = bq == a;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int c = 0; c < TC; c += 2) {
                    double v0, v1;
                    ld2(src + i * S + c, v0, v1);
                    acc[i][c] = diag ? v0 : 0.0;
                    acc[i][c + 1] = diag ? v1 : 0.0;
                }
        }
        auto step = [&](const double (&cf)[4], const double* row) __attribute__((always_inline)) {
            double rv[TC];
#pragma unroll
            for (int c = 0; c < TC; c += 2) ld2(row + c, rv[c], rv[c + 1]);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int c = 0; c < TC; ++c) acc[i][c] += cf[i] * rv[c];
        };
        if (a > 0) {  // (a > b): S_a^{-1}[i][q] G_ab[q][c]
            const double* g = gl + pidx(a, bq) * 8 * S + c0;
#pragma unroll
            for (int q = 0; q < QR; ++q) {
                double cf[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) cf[i] = Ta[(i0 + i) * S + q];
                step(cf, g + q * S);
            }
        }
        if (a < 3) {  // (b > a): G_ba[q][i] S_b^{-1}[q][c]
            const double* g = gl + pidx(bq, a) * 8 * S + i0;
            const double* Tb = Sg + bq * SS + c0;
#pragma unroll
            for (int q = 0; q < QR; ++q) {
                double cf[4];
                ld2(g + q * S, cf[0], cf[1]);
                ld2(g + q * S + 2, cf[2], cf[3]);
                step(cf, Tb + q * S);
            }
        }
#pragma unroll 1
        for (int k = a + 1; k < 4; ++k) {  // (k > a, k > b): V_ka[i][q] G_kb[q][c]
            const double* gka = gl + pidx(k, a) * 8 * S + i0;
            const double* gkb = gl + pidx(k, bq) * 8 * S + c0;
            const double* Tk = Sg + k * SS;
            double V[4][QR];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int q = 0; q < QR; ++q) V[i][q] = 0.0;
#pragma unroll
            for (int pp = 0; pp < QR; ++pp) {
                double g[4];
                ld2(gka + pp * S, g[0], g[1]);
                ld2(gka + pp * S + 2, g[2], g[3]);
#pragma unroll
                for (int q = 0; q < QR; ++q) {
                    const double t = Tk[pp * S + q];
#pragma unroll
                    for (int i = 0; i < 4; ++i) V[i][q] += g[i] * t;
                }
            }
#pragma unroll
            for (int q = 0; q < QR; ++q) {
                const double cf[4] = {V[0][q], V[1][q], V[2][q], V[3][q]};
                step(cf, gkb + q * S);
            }
        }
        // element (i0 + i, c0 + c) -> lane a 64 + (bq & 1) 32 + i0 + i, pair (jb + c0 + c) / 2
#pragma unroll
        for (int c = 0; c < TC; c += 2) {
            if (c0 + c < nbs) {
                const unsigned jp = (unsigned)((jb + c0 + c) >> 1);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    kd[jp * T4_ + t0 + i].x = acc[i][c];
                    kd[jp * T4_ + t0 + i].y = acc[i][c + 1];
                }
            }
        }
    }
}

// K: row-list length, KC: column-list length (even: the rhs splits it over the half-waves).
// factor_only: return after the first factorisation (the setup-time convexity check of
// api.hip::check_convex); the fused setup + solve kernel passes 0
// RU (the stand-alone solve kernel, k_solve_w4, not the fused setup + solve): the first
// factorisation of a solve takes setup()'s convexity factor when it is current (KParams::ffresh:
// the factor-only launch leaves the S_k^{-1} tiles in the instance's Si region, the G blocks in H
// and the eliminated columns' ec / ed in F); the factor-only launch (factor_only) persists them
// ONE (the one-shot fused kernel, mpcqp_set_one_shot; cold start): the setup left the scaled
// problem in this carve (setup_r.h ONE) and finalize stores no warm-start state -- no workspace
// round trip for data no later call reads; GL 1 (where the LDS budget of two workgroups per CU
// allows it, one_shot_form 2): the G blocks go to an LDS region after the S_k^{-1} tiles instead
// of the instance's H tiles, a refactorisation keeps y there instead of in the workspace, and
// the setup leaves E and D in the carve (edl_E / edl_D); GL 2 (one_shot_form 3): the G blocks go
// straight into gl (factorize_w4_gl)
template <int K, int KPK, int QR, bool EL = false, int KC = K, bool DK = false, bool RU = false, bool ONE = false,
          int GL = 0>
__device__ __forceinline__ void solve_w4_body(const KParams& p, double* __restrict__ xo, double* __restrict__ yo,
                                              int factor_only = 0) {
    static_assert(!(DK && EL), "the dense inverse covers plans without eliminated columns");
    const int tid = threadIdx.x, w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int h = lane >> 5, r = lane & 31;  // (rr, ch: per pass, below)
    constexpr int NB = 4, NP = NB * (NB - 1) / 2;  // exactly four blocks (solve.hip::variant_fits)
    static_assert(KC % 2 == 0, "the rhs splits the column list over the half-waves");
    constexpr int KH = KC / 2;                       // column-list entries per half in the rhs
    constexpr int LE = 2;                           // A entries of an eliminated column (plan ecnt <= 2)
    const long b = instance_of(p);
    const int n = p.n, m = p.m, npad = p.npad, nnzP = p.nnzP, nnzA = p.nnzA;
    SL2 C = carve(p);
    SLds& L = C.L;
    // GL 1: the G blocks (amax x S per pair) go to LDS after the S_k^{-1} tiles; GL 2: straight
    // into gl (factorize_w4_gl), no copy
    const double* Hg = GL == 1 ? C.L.Acsc + 2 * ((lds_base_bytes(p) + 15) / 16) + (long)NB * SS
                           : p.H + b * (long)p.nb * SS;
    double* const Sg = C.L.Acsc + 2 * ((lds_base_bytes(p) + 15) / 16);  // S_k^{-1} tiles in LDS (lds_w2_bytes)

    if (p.err[b]) {
        for (int j = tid; j < n; j += T4) if (xo) xo[b * n + j] = __builtin_nan("");
        for (int i = tid; i < m; i += T4) if (yo) yo[b * m + i] = __builtin_nan("");
        if (tid == 0) fail_status(p, b);
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
    // OPQ: the instantiations whose solve loop leaves no register for values used only at run
    // starts, refactorisations and checks (the eliminated-column and QR = 8 ones); they form
    // those values where used (see the lane identity at the top of the outer loop)
    constexpr bool OPQ = EL || QR > 5;
    // c and 1 / c of the cost scaling, from the instance's scal slots where used
    auto cscal = [&](int k) __attribute__((always_inline)) {
        return OPQ ? opaque_gptr(p.scal + b * 4)[k] : p.scal[b * 4 + k];
    };
    double rho = p.scal[b * 4 + 2];
    const double sigma = p.sigma, alpha = p.alpha;
    const bool warm = !ONE && p.warm_start != 0;
    const int mp = solve_mpad(m);
    if constexpr (!ONE) {
        for (int e = tid; e < nnzA; e += T4) L.Acsc[e] = p.Ax[b * nnzA + e];
        if (tid == 0) L.Acsc[nnzA] = 0.0;
        for (int v = tid; v < nnzP; v += T4) L.Pv[v] = p.Px[b * nnzP + v];
        if (tid == 0) L.Pv[nnzP] = 0.0;
        for (int i = tid; i < mp; i += T4) {
            const bool in = i < m;
            L.lo[i] = in ? p.l[b * m + i] : 0.0;
            L.up[i] = in ? p.u[b * m + i] : 0.0;
            L.ct[i] = in ? p.ct[b * m + i] : 0;
            C.Z[i] = (in && warm) ? p.z[b * m + i] : 0.0;
        }
        for (int pc = tid; pc < npad; pc += T4) {
            L.qv[pc] = p.q[b * npad + pc];
            C.X[pc] = warm ? p.x[b * npad + pc] : 0.0;
        }
    } else {
        if (tid == 0) L.Acsc[nnzA] = 0.0;
        if (tid == 0) L.Pv[nnzP] = 0.0;
        if constexpr (GL == 2)  // (factorize_w4_gl writes rows < amax of the pairs; the rest stays zero)
            for (int o = tid; o < (NP + 1) * 8 * S; o += T4) L.gl[o] = 0.0;
    }
    if (tid < 8) L.cor[tid] = 0.0;        // c_0 = 0 (block 0 has no correction)
    if (tid < 8) L.cor[32 + tid] = 0.0;   // the upper half's zero correction row (phase B)
    if (tid < 16) L.res[tid] = 0.0;
    if (tid < 4) L.flag[tid] = 0;

    int status = MPCQP_UNSOLVED_, rho_updates = 0, iter = 0, info_iter = 0;
    bool can_check = false, need_factor = true;
    const bool low = h == 0;
    const int pe0 = (EL && !low) ? p.eown[w * S + r] : -1;  // the upper lane's eliminated column, or -1
    const bool colv = low && p.pad_var[w * S + r] >= 0;     // a real block column (padding: rb = 0)
    double* const Fo = p.F + b * (long)p.nb * SS;    // ec, ed of the eliminated columns (factorize_w4)
    double ec = 0.0, ed = 0.0;
    const unsigned abase = lds_addr(L.Acsc), wbase = lds_addr(L.w), xbase = lds_addr(L.xt);
    const unsigned Xbase = lds_addr(C.X);
    GatherW<K> rg;
    GatherW<KH> chs;  // the half's share of the block column's list (the rhs sums)
    GatherW<LE> el;   // EL: the eliminated column's list (zero entries for the other lanes)
    const bool rows_wave = w * 64 < mp;  // wave-uniform
    // DK: the lane's half of row pc of M^{-1}: columns [0, NB0) of block h and [0, NB1) of block
    // 2 + h (their real columns), formed after each factorisation.  NB0 = 26, NB1 = 28
    // (dense_w4: bsize[0], bsize[1] <= 26 and bsize[2], bsize[3] <= 28; cfg 2's balanced
    // blocks are 26 / 25 / 25 / 28)
    constexpr int NB0 = 26, NB1 = 28;
    static_assert(!DK || (NB0 + NB1) * T4 == kDenseRowDoubles, "KParams::Kd rows");
    double Kr[DK ? NB0 + NB1 : 1];
    constexpr int DKW = 8;  // DK: b values read per batch of the product (even)
    PH(5)
    for (;;) {
        // The lane's identity through an empty asm at each pass (opaque_v): the addresses and
        // slot offsets that a refactorisation, the run start and a check form from it are
        // formed in the pass, instead of once per kernel and then held -- spilled to scratch
        // -- across the solve.  Only where the solve loop leaves no register for them (the
        // eliminated-column and QR = 8 instantiations: 42 and 17 spilled values without it,
        // none with it, cfg 3 45.5 -> 44.0 ms); the cfg-2 kernel (QR = 5) spills nothing
        // either way and is 1 % faster keeping them (same-box A/B 0.433 vs 0.439 ms).
        const int tid = OPQ ? opaque_v(threadIdx.x) : (int)threadIdx.x;
        const int lane = tid & 63, h = lane >> 5, r = lane & 31, rr = lane >> 3, ch = lane & 7;
        const int pc = w * S + r;  // the lane's column (both halves; the lower half stores)
        const int pe = OPQ ? opaque_v(pe0) : pe0;
        const int xc = pe >= 0 ? pe : pc;  // the column whose x, q the lane keeps
        const int ri = min(tid, mp - 1);   // lanes past the padded rows repeat the inert last row
        __syncthreads();
        if (need_factor) {
            need_factor = false;
            if (iter > 0) {
                if constexpr (GL == 1) {  // (y kept on chip, after the G blocks)
                    double* const ysv = Sg + (long)NB * SS + (long)(NB * (NB - 1) / 2) * p.amax * S;
                    for (int i = tid; i < m; i += T4) ysv[i] = L.ys[i];
                } else {
                    const auto yp = opaque_gptr(p.y + b * m);
                    for (int i = tid; i < m; i += T4) yp[i] = L.ys[i];
                }
                __syncthreads();  // every ys read is done before factorize_w4's E tiles overwrite it
            }
            // the slack layouts' (EL) factorisation with rotated tile rows: cfg 3
            // 43.38 -> 43.16 ms; cfg 2's build lost 1.6 % to the register assignment it moved
            // (profiles/r3s3_ab/ab_swz*.json)
            bool ok;
            if constexpr (RU) {
                // the workspace factor is setup()'s (same data, rho and row classes: the same
                // arithmetic, so the same tiles) -- used once: this solve's later factorisations,
                // and the ones of later solves, are its own
                if (iter == 0 && p.reuse && p.ffresh[b] == 1 && p.scal[b * 4 + 3] == rho) {
                    const double2* src = (const double2*)(p.Si + b * (long)p.nb * SS);
                    for (int e = tid; e < 2 * SS; e += T4) ((double2*)Sg)[e] = src[e];
                    ok = true;
                } else if constexpr (EL) {
                    ok = factorize_lds_nl<T4, EL>(p.self, b, rho);
                } else {
                    ok = factorize_nl<T4, EL>(p.self, b, rho, Sg);
                }
                __syncthreads();
                if (tid == 0) p.ffresh[b] = 0;
            } else if constexpr (GL == 1) {
                ok = factorize_g_nl<T4, EL>(p.self, b, rho);
            } else if constexpr (GL == 2) {
                ok = factorize_gl_nl<T4, EL>(p.self, b, rho);
            } else if constexpr (EL) {
                // (the tiles from the carve: an LDS-typed pointer, ds_ accesses -- cfg 3's
                // factorisation was compiled with flat ones)
                ok = factorize_lds_nl<T4, EL>(p.self, b, rho);
            } else {
                ok = factorize_nl<T4, EL>(p.self, b, rho, Sg);
            }
            if (!ok) {
                if (iter == 0) {
                    if (xo) for (int j = tid; j < n; j += T4) opaque_ptr(xo + b * n)[j] = __builtin_nan("");
                    if (yo) for (int i = tid; i < m; i += T4) opaque_ptr(yo + b * m)[i] = __builtin_nan("");
                    if (tid == 0) fail_status(p, b);
                    return;
                }
                status = MPCQP_NON_CVX_;
                can_check = true;
                break;
            }
            if (factor_only) {  // (setup()'s convexity check: its tiles for the first solve, RU)
                __syncthreads();
                double2* dst = (double2*)(p.Si + b * (long)p.nb * SS);
                for (int e = tid; e < 2 * SS; e += T4) dst[e] = ((const double2*)Sg)[e];
                if (tid == 0) {
                    p.ffresh[b] = 1;
                    p.scal[b * 4 + 3] = rho;  // the factor's rho (the RU solve checks it against scal[2])
                }
                return;
            }
            __syncthreads();
            const bool have_y = iter > 0 || warm;
            if constexpr (GL == 1) {
                const double* const ysv = Sg + (long)NB * SS + (long)(NB * (NB - 1) / 2) * p.amax * S;
                for (int i = tid; i < mp; i += T4) L.ys[i] = (have_y && i < m) ? ysv[i] : 0.0;
            } else {
                const auto yp = opaque_gptr(p.y + b * m);
                for (int i = tid; i < mp; i += T4) L.ys[i] = (have_y && i < m) ? yp[i] : 0.0;
            }
            if constexpr (GL != 2) {
                for (int o = tid; o < (NP + 1) * 8 * S; o += T4) {
                    const int q = o >> 8, t = (o >> 5) & 7;
                    L.gl[o] = (q < NP && t < p.amax) ? Hg[(long)q * p.amax * S + (o & 255)] : 0.0;
                }
            }
            chs.load(p.gcol + (h ? KH : 0) * npad + pc, npad, abase, wbase);
            if constexpr (EL) {
                if (pe >= 0) {
                    el.load(p.gcol + pe, npad, abase, wbase);
                    const int e = pe - p.nb * S;
                    ec = Fo[2 * e];
                    ed = Fo[2 * e + 1];
                } else {
                    el.clear(abase + 8u * nnzA, wbase);
                }
            }
            if (ri < m) rg.load(p.grow + ri, m, abase, xbase);  // by ri: duplicate lanes repeat its row
            else rg.clear(abase + 8u * nnzA, xbase);
            if constexpr (DK) {
                // M^{-1}'s rows formed once per factorisation and kept in the instance's Kd rows
                // (lane-contiguous pairs): each run start reloads them, so that nothing lives in
                // registers across the termination check -- the check's registers and the
                // 108 of the rows do not fit together (spilled, and wrong in the divergent
                // check: DESIGN.md §5)
                __syncthreads();  // the G copy is complete
                // (the instance's base through an empty asm, the lanes' 32-bit indices formed at
                // the stores; the run start's reads follow a workgroup barrier)
                form_dense_rows<QR, NB0, NB1>((__attribute__((address_space(1))) dpair*)opaque_gptr(
                                                  p.Kd + b * kDenseRowDoubles),
                                              Sg, L.gl, w, lane);
                __syncthreads();  // every tile stored before any lane reads its rows (run start)
            }
            PH(0)
        }
        // ---- run state ----
        if constexpr (DK) {
            const auto kd = (const __attribute__((address_space(1))) dpair*)opaque_gptr(p.Kd + b * kDenseRowDoubles);
#pragma unroll
            for (int j = 0; j < NB0 + NB1; j += 2) {
                Kr[j] = kd[(unsigned)((j / 2) * T4 + tid)].x;
                Kr[j + 1] = kd[(unsigned)((j / 2) * T4 + tid)].y;
            }
        }
        double SB[16];
        if constexpr (!DK) {
            const double* src = Sg + (long)w * SS + r * S + 16 * h;
#pragma unroll
            for (int c = 0; c < 16; c += 2) ld2(src + c, SB[c], SB[c + 1]);
        }
        double X = C.X[xc], DX = 0.0;
        const double Q = L.qv[xc];
        // phase-C slots: pairs (j, w), j > w, split over the halves; pair NP is zero
        int gslot[2], tslot[2];
        {
            int pr[2] = {NP, NP}, jj[2] = {3, 3};
            if (w == 0) {
                if (h == 0) { pr[0] = 0; jj[0] = 1; pr[1] = 1; jj[1] = 2; }
                else        { pr[0] = 3; jj[0] = 3; }
            } else if (w == 1) {
                if (h == 0) { pr[0] = 2; jj[0] = 2; }
                else        { pr[0] = 4; jj[0] = 3; }
            } else if (w == 2) {
                if (h == 0) { pr[0] = 5; jj[0] = 3; }
            }
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                gslot[s] = lds_addr(L.gl + pr[s] * 8 * S + r);
                tslot[s] = lds_addr(L.tv + jj[s] * 8);
            }
        }
        const int nsw = (NB - w) >> 1;  // phase-C slots of the wave (wave 0: 2, waves 1-2: 1, wave 3: 0)
        // the half's share of the column list (KH entries; the list is zero-padded to K)
        const GatherW<KH>& ch2 = chs;
        double ca[KH];  // the half's A values of the column (registers for the run)
#pragma unroll
        for (int k = 0; k < KH; ++k) ca[k] = lds_at(ch2.e[k] & 0xFFFFu);
        double ea[LE];  // EL: the eliminated column's A values (zeros on the other lanes)
#pragma unroll
        for (int k = 0; k < LE; ++k) ea[k] = EL ? lds_at(el.e[k] & 0xFFFFu) : 0.0;
        double bj = 0.0;  // EL: b of the eliminated column, from the rhs to phase C
        const double r_hi = RHO_EQ_OVER_RHO_INEQ * rho;
        double y = L.ys[ri], Z = C.Z[ri], dy = 0.0;
        // the row's A values and bounds stay in registers for the run (fewer LDS reads per
        // iteration)
        double av[K];
#pragma unroll
        for (int k = 0; k < K; ++k) av[k] = DK ? 0.0 : lds_at(rg.e[k] & 0xFFFFu);
        const double rlo = L.lo[ri], rup = L.up[ri];
        const signed char cl = L.ct[ri];
        const double rv = cl < 0 ? RHO_MIN : (cl > 0 ? r_hi : rho);
        const double rvi = cl < 0 ? 1.0 / RHO_MIN : (cl > 0 ? 1.0 / r_hi : 1.0 / rho);
        __syncthreads();  // (the G copy of a refactorisation is complete)
        // phase A's G values (rows rr < 8 of G_wj, columns [4 ch, 4 ch + 4), j < w) in registers for the run
        double ga[NB - 1][4];
        if constexpr (!DK) {
            const double* gq = L.gl + (w * (w - 1) / 2) * 8 * S + rr * S + 4 * ch;
#pragma unroll
            for (int j = 0; j < NB - 1; ++j) {
                if (j < w) {
                    ld2(gq + j * 8 * S, ga[j][0], ga[j][1]);
                    ld2(gq + j * 8 * S + 2, ga[j][2], ga[j][3]);
                } else {
                    ga[j][0] = ga[j][1] = ga[j][2] = ga[j][3] = 0.0;
                }
            }
        }
        // phase C's G values (column r of the slots' pairs, rows < QR) in registers for the run
        double gc[2][QR];
        if constexpr (!DK) {
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int q = 0; q < QR; ++q) gc[s][q] = s < nsw ? lds_at(gslot[s] + q * S * 8) : 0.0;
        }
        if (rows_wave) L.w[ri] = rv * Z - y;  // (lanes past the padded rows may hold a stale y)
        int stop_at = p.max_iter;
        if (p.check_term) stop_at = min(stop_at, (iter / p.check_term + 1) * p.check_term);
        if (p.adaptive_rho && p.rho_interval) stop_at = min(stop_at, (iter / p.rho_interval + 1) * p.rho_interval);
        __syncthreads();
        PH(5)
        double* const cw = L.cor + w * 8;                 // c_w rows < 8
        const double* const cwh = L.cor + (h ? 32 : w * 8);  // the half's correction (upper half: zeros)
        while (iter < stop_at) {
            ++iter;
            // rhs = sigma x_prev - q + A' (rho z_prev - y), column pc: the lower half sums
            // the list's first KH entries, the upper half the rest, one permlane32 swap
            {
                double wv[KH];
#pragma unroll
                for (int k = 0; k < KH; ++k) wv[k] = lds_at(ch2.e[k] >> 16);
                double v;
                if constexpr (EL) {
                    // sigma x - q of the lane's column (upper: the eliminated one, whose list it
                    // adds; zero entries on the other lanes), then the upper half's b_p share
                    // carries -ec b_pe
                    double we[LE];
#pragma unroll
                    for (int k = 0; k < LE; ++k) we[k] = lds_at(el.e[k] >> 16);
                    bj = sigma * X - Q;
#pragma unroll
                    for (int k = 0; k < LE; ++k) bj += ea[k] * we[k];
                    v = low ? bj : -(ec * bj);
                } else {
                    v = low ? sigma * X - Q : 0.0;
                }
#pragma unroll
                for (int k = 0; k < KH; ++k) v += ca[k] * wv[k];
                const unsigned vlo = (unsigned)__double2loint(v), vhi = (unsigned)__double2hiint(v);
                const auto l2 = __builtin_amdgcn_permlane32_swap(vlo, vlo, false, false);
                const auto h2 = __builtin_amdgcn_permlane32_swap(vhi, vhi, false, false);
                const double v0 = __hiloint2double((int)h2[0], (int)l2[0]);
                const double v1 = __hiloint2double((int)h2[1], (int)l2[1]);
                if (low) L.rb[pc] = colv ? v0 + v1 : 0.0;
            }
            __syncthreads();
            PH(1)
            if constexpr (DK) {
                // x~[pc] = M^{-1}[pc] b: the half's NB0 + NB1 columns (broadcast reads, one address
                // per half-wave), four FMA chains, one permlane32 swap
                const double* const rbh = L.rb + S * h;
                double a[4] = {0.0, 0.0, 0.0, 0.0};
                // software-pipelined in windows of DKW values: window k + 1's reads are issued
                // before window k's FMAs (two windows in flight; all 27 reads at once spill)
                constexpr int NE = NB0 + NB1, NWIN = (NE + DKW - 1) / DKW;
                double v[2][DKW];
                auto issue = [&](int k, double (&dst)[DKW]) __attribute__((always_inline)) {
#pragma unroll
                    for (int c = 0; c < DKW; c += 2) {
                        const int e = k * DKW + c;  // block h column e, or block 2 + h column e - NB0
                        if (e < NE) ld2(rbh + (e < NB0 ? e : 2 * S + e - NB0), dst[c], dst[c + 1]);
                    }
                };
                issue(0, v[0]);
#pragma unroll
                for (int k = 0; k < NWIN; ++k) {
                    if (k + 1 < NWIN) issue(k + 1, v[(k + 1) & 1]);
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int c = 0; c < DKW; ++c)
                        if (k * DKW + c < NE) a[c & 3] += Kr[k * DKW + c] * v[k & 1][c];
                    __builtin_amdgcn_sched_barrier(0);
                }
                const double th = (a[0] + a[1]) + (a[2] + a[3]);
                const unsigned lo = (unsigned)__double2loint(th), hi = (unsigned)__double2hiint(th);
                const auto l2 = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
                const auto h2 = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
                const double xn = __hiloint2double((int)h2[0], (int)l2[0]) + __hiloint2double((int)h2[1], (int)l2[1]);
                if (low) L.xt[pc] = xn;
                const double xnew = alpha * xn + (1.0 - alpha) * X;
                DX = xnew - X;
                X = xnew;
            } else {
            // A: c_w = sum_{j<w} G_wj b_j (rows < 8), wave w only
            if (w > 0) {
                // one accumulator per pair (wave 3: three 4-deep FMA chains instead of one 12-deep)
                double acc[NB - 1] = {0.0, 0.0, 0.0};
#pragma unroll
                for (int j = 0; j < NB - 1; ++j) {
                    if (j < w) {
                        double bj[4];
                        ld2(L.rb + j * S + 4 * ch, bj[0], bj[1]);
                        ld2(L.rb + j * S + 4 * ch + 2, bj[2], bj[3]);
#pragma unroll
                        for (int e = 0; e < 4; ++e) acc[j] += ga[j][e] * bj[e];
                    }
                }
                cw[rr] = reduce8((acc[0] + acc[1]) + acc[2]);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            PH(12)
            // B: t_w[r] = S_w^{-1}[r] (b_w + c_w): half-row sums, permlane32 swap
            double t;
            {
                constexpr int QE = (QR + 1) & ~1;  // c_w's nonzero rows (< amax), read in pairs
                double v[16], cc[QE];
#pragma unroll
                for (int c = 0; c < 16; c += 2) ld2(L.rb + w * S + 16 * h + c, v[c], v[c + 1]);
#pragma unroll
                for (int c = 0; c < QE; c += 2) ld2(cwh + c, cc[c], cc[c + 1]);
#pragma unroll
                for (int c = 0; c < QR; ++c) v[c] += cc[c];
                double a[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int c = 0; c < 16; ++c) a[c & 3] += SB[c] * v[c];
                const double th = (a[0] + a[1]) + (a[2] + a[3]);
                const unsigned lo = (unsigned)__double2loint(th), hi = (unsigned)__double2hiint(th);
                const auto l2 = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
                const auto h2 = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
                const double t0 = __hiloint2double((int)h2[0], (int)l2[0]);  // lower half's
                const double t1 = __hiloint2double((int)h2[1], (int)l2[1]);  // upper half's
                t = t0 + t1;
                if (low && r < 8) L.tv[w * 8 + r] = t;
            }
            __syncthreads();
            PH(13)
            // C: x~_w[r] = t + sum_s G_{pair_s}[q][r] t_{j_s}[q]  (slots split over the halves;
            // rows q < QR: the G blocks are zero from row amax on)
            {
                constexpr int QE = (QR + 1) & ~1;  // t rows read in pairs
                // the wave's slot count (wave 0: 2, waves 1-2: 1, wave 3: 0): slots no half
                // of the wave has a pair for are skipped, not read as the zero pair (LDS
                // return bandwidth is shared with the CU's other workgroup)
                double gv[2][QE], tq[2][QE];
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    if (s < nsw) {
#pragma unroll
                        for (int q = 0; q < QE; ++q) gv[s][q] = q < QR ? gc[s][q] : 0.0;
#pragma unroll
                        for (int q = 0; q < QE; q += 2) lds_at2(tslot[s] + q * 8, tq[s][q], tq[s][q + 1]);
                    } else {
#pragma unroll
                        for (int q = 0; q < QE; ++q) gv[s][q] = tq[s][q] = 0.0;
                    }
                }
                double a0 = 0.0, a1 = 0.0;
#pragma unroll
                for (int s = 0; s < 2; ++s)
#pragma unroll
                    for (int q = 0; q < QR; q += 2) {
                        a0 += gv[s][q] * tq[s][q];
                        if (q + 1 < QR) a1 += gv[s][q + 1] * tq[s][q + 1];
                    }
                const double d = a0 + a1;
                const unsigned lo = (unsigned)__double2loint(d), hi = (unsigned)__double2hiint(d);
                const auto l2 = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
                const auto h2 = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
                const double d0 = __hiloint2double((int)h2[0], (int)l2[0]);
                const double d1 = __hiloint2double((int)h2[1], (int)l2[1]);
                const double xn = t + (d0 + d1);
                if (low) L.xt[pc] = xn;
                double xl = xn;  // x~ of the lane's column
                if constexpr (EL) {
                    if (!low) {
                        xl = ed * bj - ec * xn;
                        if (pe >= 0) L.xt[pe] = xl;
                    }
                }
                const double xnew = alpha * xl + (1.0 - alpha) * X;
                DX = xnew - X;
                X = xnew;
            }
            }  // !DK
            __syncthreads();
            PH(14)
            // rows: z~ = A x~ ; relaxed + projected z ; y ; next w (waves wholly past the
            // padded rows skip it: their lanes would only repeat the inert last row)
            if (rows_wave) {
                double xv[K], ar[K];
#pragma unroll
                for (int k = 0; k < K; ++k) xv[k] = lds_at(rg.e[k] >> 16);
                // DK: the row's A values read with x~ (the dense rows leave no registers to
                // keep them across the run)
#pragma unroll
                for (int k = 0; k < K; ++k) ar[k] = DK ? lds_at(rg.e[k] & 0xFFFFu) : av[k];
                const double lo = rlo, up = rup;
                double zt = ar[0] * xv[0];
#pragma unroll
                for (int k = 1; k < K; ++k) zt += ar[k] * xv[k];
                const double zr = alpha * zt + (1.0 - alpha) * Z;
                const double zn = __builtin_fmin(__builtin_fmax(zr + rvi * y, lo), up);
                const double dd = rv * (zr - zn);
                Z = zn;
                dy = dd;
                y += dd;
                L.w[ri] = rv * zn - y;
            }
            __syncthreads();
            PH(3)
        }
        // run state back to LDS (lds_put: the addresses are formed here, not held across the
        // loop)
        if (low) { lds_put(C.X, pc, X); lds_put(L.dx, pc, DX); }
        if (EL && pe >= 0) { lds_put(C.X, pe, X); lds_put(L.dx, pe, DX); }
        if (rows_wave) { lds_put(L.ys, ri, y); lds_put(C.Z, ri, Z); lds_put(C.dY, ri, dy); }
        __syncthreads();
        can_check = p.check_term && (iter % p.check_term == 0);
        const bool do_rho = p.adaptive_rho && p.rho_interval && (iter % p.rho_interval == 0);
        if (!can_check && !do_rho) break;
        info_iter = iter;
        bool stop = false;
        {
            // the check's per-lane operands come from the plan (shared by every instance: L2
            // hits) and the workspace here, not from registers held through the run: the lane's
            // column (EL: the upper half checks its eliminated column pe) with its A and P lists
            // and D, the row's E
            const int col = EL ? (low ? pc : pe) : pc;
            const bool cv = col >= 0 && (EL || low) && opaque_gptr(p.pad_var)[col] >= 0;
            GatherW<KC> cg;
            GatherW<KPK> pg;
            if (col >= 0) {
                cg.load(p.gcol + col, npad, abase, wbase);
                pg.load(p.gpsym + col, npad, lds_addr(L.Pv), Xbase);
            } else {
                cg.clear(abase + 8u * nnzA, wbase);
                pg.clear(lds_addr(L.Pv) + 8u * nnzP, Xbase);
            }
            const int oz = opaque_zero();
            double Dv, Ev;
            if constexpr (GL == 1) {  // (E and D on chip: the one-shot form 2, edl_E / edl_D)
                Dv = col >= 0 ? edl_D(p, C)[col] : 1.0;
                Ev = ri < m ? edl_E(p, C)[ri] : 1.0;
            } else {
                Dv = col >= 0 ? opaque_gptr(p.D + b * npad)[col] : 1.0;
                Ev = ri < m ? opaque_gptr(p.E + b * m)[ri] : 1.0;
            }
            // inline update_info + check_termination (as solve_w2_body's), one row per thread
            const bool unscale = p.scaling && !p.scaled_term;
            const unsigned ysbase = lds_addr(L.ys), dYbase = lds_addr(C.dY), dxbase = lds_addr(L.dx);
            double mx[17], sm[2] = {0.0, 0.0}, adx = 0.0;
#pragma unroll
            for (int k = 0; k < 17; ++k) mx[k] = 0.0;
            {
                const bool ok = tid < m;
                double ax = 0.0, ad = 0.0;
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const unsigned e = rg.e[k], va = e >> 16;
                    const double a = lds_at(e & 0xFFFFu);
                    ax += a * lds_at(va - xbase + Xbase);
                    ad += a * lds_at(va - xbase + dxbase);
                }
                adx = ad;
                const double zi = Z, pr = ax - zi, ei = 1.0 / Ev;
                const double lo = L.lo[ri], up = L.up[ri];
                double d = dy;
                if (up > OSQP_INFTY * MIN_SCALING) d = (lo < -OSQP_INFTY * MIN_SCALING) ? 0.0 : cmin(d, 0.0);
                else if (lo < -OSQP_INFTY * MIN_SCALING) d = cmax(d, 0.0);
                if (ok) {
                    mx[0] = fabs(ei * pr);
                    mx[2] = fabs(ei * zi);
                    mx[3] = fabs(ei * ax);
                    mx[7] = fabs(pr);
                    mx[9] = fabs(zi);
                    mx[10] = fabs(ax);
                    mx[14] = fabs(unscale ? Ev * d : d);
                    sm[0] = up * cmax(d, 0.0) + lo * cmin(d, 0.0);
                    C.dY[ri] = d;
                }
            }
            {  // the lane's column (lower half): P x, A' y, P dx, and the delta x norm
                double px = 0.0, pdx = 0.0, aty = 0.0;
#pragma unroll
                for (int k = 0; k < KPK; ++k) {
                    const unsigned e = pg.e[k], va = e >> 16;
                    const double pv = lds_at(e & 0xFFFFu);
                    px += pv * lds_at(va);
                    pdx += pv * lds_at(va - Xbase + dxbase);
                }
#pragma unroll
                for (int k = 0; k < KC; ++k) {
                    const unsigned e = cg.e[k];
                    aty += lds_at(e & 0xFFFFu) * lds_at((e >> 16) - wbase + ysbase);
                }
                if (cv) {
                    const double d = (Q + px) + aty, di = 1.0 / Dv;
                    mx[1] = fabs(di * d);
                    mx[4] = fabs(di * Q);
                    mx[5] = fabs(di * aty);
                    mx[6] = fabs(di * px);
                    mx[8] = fabs(d);
                    mx[11] = fabs(Q);
                    mx[12] = fabs(aty);
                    mx[13] = fabs(px);
                    mx[15] = fabs(unscale ? Dv * DX : DX);
                    mx[16] = fabs(unscale ? pdx * di : pdx);
                }
            }
            if (tid < npad && opaque_gptr(p.pad_var)[tid] >= 0) sm[1] = L.qv[tid + oz] * L.dx[tid + oz];
            if (do_rho || !unscale) {
                block_max_sum_tr<T4, 17, 2>(mx, sm, L.red);
            } else {
                // a check that adapts no rho decides with the unscaled norms and the
                // certificates' only: 10 maxima instead of 17 (R's scaled norms are then stale
                // and unread: only a rho step restores them)
                double m10[10] = {mx[0], mx[1], mx[2], mx[3], mx[4], mx[5], mx[6], mx[14], mx[15], mx[16]};
                block_max_sum_tr<T4, 10, 2>(m10, sm, L.red);
#pragma unroll
                for (int k = 0; k < 7; ++k) mx[k] = m10[k];
                mx[14] = m10[7];
                mx[15] = m10[8];
                mx[16] = m10[9];
            }
            Res R;
            if (unscale) {
                R.pri = mx[0]; R.dua = cscal(1) * mx[1];
                R.nz = mx[2]; R.nax = mx[3]; R.nq = mx[4]; R.naty = mx[5]; R.npx = mx[6];
            } else {
                R.pri = mx[7]; R.dua = mx[8];
                R.nz = mx[9]; R.nax = mx[10]; R.nq = mx[11]; R.naty = mx[12]; R.npx = mx[13];
            }
            R.rpri = mx[7]; R.rdua = mx[8]; R.rz = mx[9]; R.rax = mx[10]; R.rq = mx[11]; R.raty = mx[12]; R.rpx = mx[13];
            if (m == 0) R.pri = 0.0;
            if (tid == 0) R.save(L.res);
            if (can_check) {
                int st = MPCQP_UNSOLVED_;
                bool done = false;
                if (R.pri > OSQP_INFTY || R.dua > OSQP_INFTY) {
                    st = MPCQP_NON_CVX_;
                    done = true;
                } else {
                    const bool prim_ok = m == 0 || R.pri < p.eps_abs + p.eps_rel * cmax(R.nz, R.nax);
                    double mxd = cmax(cmax(R.nq, R.naty), R.npx);
                    if (unscale) mxd *= cscal(1);
                    const bool dual_ok = R.dua < p.eps_abs + p.eps_rel * mxd;
                    bool prim_inf = false, dual_inf = false;
                    if (!prim_ok || !dual_ok) {
                        const double norm_dy = mx[14], norm_dx = mx[15], epi = p.eps_pinf, edi = p.eps_dinf;
                        const double cs = unscale ? cscal(0) : 1.0;
                        if (!prim_ok && m != 0 && norm_dy > epi && sm[0] < epi * norm_dy) {
                            __syncthreads();
                            double na[1] = {0.0};
                            double a = 0.0;
#pragma unroll
                            for (int k = 0; k < KC; ++k) {
                                const unsigned e = cg.e[k];
                                a += lds_at(e & 0xFFFFu) * lds_at((e >> 16) - wbase + dYbase);
                            }
                            if (cv) na[0] = fabs(unscale ? a * (1.0 / Dv) : a);
                            block_max<T4, 1>(na, L.red);
                            prim_inf = na[0] < epi * norm_dy;
                        }
                        if (!dual_ok && norm_dx > edi && sm[1] < cs * edi * norm_dx && mx[16] < cs * edi * norm_dx) {
                            bool viol = false;
                            if (tid < m) {
                                const double ar = unscale ? adx * (1.0 / Ev) : adx;
                                const double lo = L.lo[ri], up = L.up[ri];
                                if ((up < OSQP_INFTY * MIN_SCALING && ar > edi * norm_dx) ||
                                    (lo > -OSQP_INFTY * MIN_SCALING && ar < -edi * norm_dx))
                                    viol = true;
                            }
                            dual_inf = !block_any<T4>(viol, L.flag);
                        }
                    }
                    if (prim_ok && dual_ok) {
                        st = MPCQP_SOLVED_;
                        done = true;
                    } else if (prim_inf) {
                        st = MPCQP_PRIMAL_INFEASIBLE_;
                        if (tid == 0) L.flag[3] = unscale;
                        done = true;
                    } else if (dual_inf) {
                        st = MPCQP_DUAL_INFEASIBLE_;
                        if (tid == 0) L.flag[2] = unscale;
                        done = true;
                    }
                }
                __syncthreads();
                // (the objective of an infeasible / non-convex status is set by finalize_ph)
                if (done && tid == 0) L.flag[1] = st;
                __syncthreads();
                status = done ? st : MPCQP_UNSOLVED_;
                stop = done;
            }
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
    const double cval = cscal(0), cinv = cscal(1);
    if (!can_check && status == MPCQP_UNSOLVED_) {
        update_info_nl<T4, GL == 1>(p.self, b, cinv);
        info_iter = iter;
        status = check_termination_nl<T4, GL == 1>(p.self, b, cval, cinv, 0);
    }
    const bool has_sol = !(status == MPCQP_PRIMAL_INFEASIBLE_ || status == MPCQP_PRIMAL_INFEASIBLE_INACCURATE_ ||
                           status == MPCQP_DUAL_INFEASIBLE_ || status == MPCQP_DUAL_INFEASIBLE_INACCURATE_ ||
                           status == MPCQP_NON_CVX_);
    if (has_sol) objective_nl<T4>(p.self, cinv);
    if (status == MPCQP_UNSOLVED_) {
        status = check_termination_nl<T4, GL == 1>(p.self, b, cval, cinv, 1);
        if (status == MPCQP_UNSOLVED_) status = MPCQP_MAX_ITER_REACHED_;
    }
    finalize_nl<T4, ONE, GL == 1>(p.self, b, xo, yo, cinv, rho, status, info_iter, rho_updates, p.ostat, p.oiter);
#ifdef MPCQP_PHASE_PROF
    if (prof) {
        __syncthreads();
        PH(5)
        if (tid == 0) {
#pragma unroll
            for (int k = 0; k < 6; ++k) p.prof[b * kProfSlots + k] = L.pacc[k];
#pragma unroll
            for (int k = 8; k < 15; ++k) p.prof[b * kProfSlots + k] = L.pacc[k];
            p.prof[b * kProfSlots + 2] = L.pacc[12] + L.pacc[13] + L.pacc[14];
            p.prof[b * kProfSlots + 6] = clock64() - t0c;
            p.prof[b * kProfSlots + 7] = wall_clock64() - t0w;
            p.prof[b * kProfSlots + 15] = t0w;
        }
    }
#endif
#undef PH
}

// FO: the factor-only instantiation (api.hip::check_convex), so that the solve's own code
// carries no factor_only test
template <int K, int KPK, int QR, bool EL = false, int KC = K, bool FO = false, bool DK = false>
__global__ __launch_bounds__(T4, 2) void k_solve_w4(KParams p, double* __restrict__ xo, double* __restrict__ yo,
                                                    int /*factor_only: FO*/) {
    solve_w4_body<K, KPK, QR, EL, KC, DK, !FO && !DK>(p, xo, yo, FO ? 1 : 0);
    extern __shared__ __attribute__((aligned(16))) double sm[];
    order_epilogue<T4>(p, (int*)sm);
}

// setup (setup_r.h with 256 threads: one column and one row per thread) + solve; ONE: the
// one-shot form (solve_w4_body)
template <int K, int KPK, int QR, int SK, int SAS, bool EL = false, int KC = K, bool DK = false, bool ONE = false,
          int GL = 0>
__global__ __launch_bounds__(T4, 2) void k_setup_solve_w4(KParams p, const double* __restrict__ Px_in,
                                                          const double* __restrict__ Ax_in,
                                                          const double* __restrict__ q_in,
                                                          const double* __restrict__ l_in,
                                                          const double* __restrict__ u_in, double* __restrict__ xo,
                                                          double* __restrict__ yo) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    setup_r_body<T4, SK, 4, 1, SAS, 1, false, ONE, GL == 1>(p, instance_of(p), Px_in, Ax_in, q_in, l_in, u_in, sm);
    __syncthreads();
    solve_w4_body<K, KPK, QR, EL, KC, DK, false, ONE, GL>(p, xo, yo);
    order_epilogue<T4>(p, (int*)sm);
}


#ifdef MPCQP_EXPERIMENTAL  // the eight-wave kernel (variant 18): make exp / MPCQP_BUILD=exp
// ---------------------------------------------------------------------------
// Eight-wave variant (variant 18, k_solve_w8): the four-wave kernel's iteration for nb = 8
// plans (the slack-variable MPC, SURVEY.md configs[2]/[3]): one 512-thread workgroup per
// QP, wave k owns block k (lane (h, r): row r of S_k^{-1}, columns [16 h, 16 h + 16)), one
// workgroup per CU.  The 28 G blocks (rows < 12) and the eight S_k^{-1} tiles do not fit
// in LDS together, so the tiles live only during the factorisation: S^{-1} stays in
// registers for the whole solve and the G copy reuses the tiles' LDS (solve_phases.h::
// w8_toff).  Phase A: 16 rows x 4 lanes of 8 columns per wave; phase C: up to four pairs
// per half.  MPCQP_VARIANT=18.
constexpr int T8 = 512;

template <int K, int KPK>
__device__ __forceinline__ void solve_w8_body(const KParams& p, double* __restrict__ xo, double* __restrict__ yo,
                                              int factor_only) {
    const int tid = threadIdx.x, w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int h = lane >> 5, r = lane & 31, rr = lane >> 2, ch = lane & 3;
    constexpr int NB = 8, NP = NB * (NB - 1) / 2;  // exactly eight blocks (solve.hip::variant_fits)
    constexpr int QR = 12, GR = 12;                 // G rows summed (amax <= 12) / per pair in gl
    static_assert(K % 2 == 0, "the rhs splits the column list over the half-waves");
    constexpr int KH = K / 2;                       // column-list entries per half in the rhs
    const long b = instance_of(p);
    const int n = p.n, m = p.m, npad = p.npad, nnzP = p.nnzP, nnzA = p.nnzA;
    SL2 C = carve(p);
    SLds& L = C.L;
    double* const Hg = p.H + b * (long)p.nb * SS;
    double* const Fg = p.F + b * (long)p.nb * SS;  // the G pairs past H's room (w8_gpair)
    double* const Sg = L.SP + w8_toff(p.amax);                    // S_k^{-1} tiles (in V, past the factor scratch)
    double* const red8 = L.SP + w8_roff(p.m, p.npad, p.amax);     // the inline check's reduction buffer

    if (p.err[b]) {
        for (int j = tid; j < n; j += T8) if (xo) xo[b * n + j] = __builtin_nan("");
        for (int i = tid; i < m; i += T8) if (yo) yo[b * m + i] = __builtin_nan("");
        if (tid == 0) fail_status(p, b);
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
    for (int e = tid; e < nnzA; e += T8) L.Acsc[e] = p.Ax[b * nnzA + e];
    if (tid == 0) L.Acsc[nnzA] = 0.0;
    for (int v = tid; v < nnzP; v += T8) L.Pv[v] = p.Px[b * nnzP + v];
    if (tid == 0) L.Pv[nnzP] = 0.0;
    const int mp = solve_mpad(m);
    for (int i = tid; i < mp; i += T8) {
        const bool in = i < m;
        L.lo[i] = in ? p.l[b * m + i] : 0.0;
        L.up[i] = in ? p.u[b * m + i] : 0.0;
        L.ct[i] = in ? p.ct[b * m + i] : 0;
        C.Z[i] = (in && warm) ? p.z[b * m + i] : 0.0;
    }
    for (int pc = tid; pc < npad; pc += T8) {
        L.qv[pc] = p.q[b * npad + pc];
        C.X[pc] = warm ? p.x[b * npad + pc] : 0.0;
    }
    if (tid < 16) L.cor[tid] = 0.0;        // c_0 = 0 (block 0 has no correction)
    if (tid < 16) L.cor[128 + tid] = 0.0;  // the upper half's zero correction row (phase B)
    if (tid < 16) L.res[tid] = 0.0;
    if (tid < 4) L.flag[tid] = 0;

    int status = MPCQP_UNSOLVED_, rho_updates = 0, iter = 0, info_iter = 0;
    bool can_check = false, need_factor = true;
    const int pc = w * S + r;  // the lane's column (both halves; the lower half stores)
    const bool low = h == 0;
    const unsigned abase = lds_addr(L.Acsc), wbase = lds_addr(L.w), xbase = lds_addr(L.xt);
    const unsigned Xbase = lds_addr(C.X);
    bool cv = false;
    double Dv = 1.0, Ev = 1.0;
    GatherW<K> cg, rg;
    GatherW<KPK> pg;
    const int ri = min(tid, mp - 1);  // lanes past the padded rows repeat the inert last row
    const bool rows_wave = w * 64 < mp;  // wave-uniform: waves wholly past the padded rows skip the rows
    double SB[16];                    // row r of S_w^{-1}, columns [16 h, 16 h + 16): kept across runs
#pragma unroll
    for (int c = 0; c < 16; ++c) SB[c] = 0.0;
    PH(5)
    for (;;) {
        __syncthreads();
        if (need_factor) {
            need_factor = false;
            if (iter > 0) {
                for (int i = tid; i < m; i += T8) p.y[b * m + i] = L.ys[i];
                __syncthreads();  // every ys read is done before factorize_w4's E tiles overwrite it
            }
            const bool ok = factorize_nl<T8>(p.self, b, rho, Sg);
            if (!ok) {
                if (iter == 0) {
                    for (int j = tid; j < n; j += T8) if (xo) xo[b * n + j] = __builtin_nan("");
                    for (int i = tid; i < m; i += T8) if (yo) yo[b * m + i] = __builtin_nan("");
                    if (tid == 0) fail_status(p, b);
                    return;
                }
                status = MPCQP_NON_CVX_;
                can_check = true;
                break;
            }
            if (factor_only) return;
            __syncthreads();
            {
                const double* src = Sg + (long)w * SS + r * S + 16 * h;
#pragma unroll
                for (int c = 0; c < 16; c += 2) ld2(src + c, SB[c], SB[c + 1]);
            }
            __syncthreads();  // the tiles are in registers: the G copy overwrites them
            const bool have_y = iter > 0 || warm;
            for (int i = tid; i < mp; i += T8) L.ys[i] = (have_y && i < m) ? p.y[b * m + i] : 0.0;
            for (int o = tid; o < (NP + 1) * GR * S; o += T8) {
                const int q = o / (GR * S), t = (o >> 5) - q * GR;
                L.gl[o] = (q < NP && t < p.amax) ? w8_gpair(Fg, Hg, p.amax, q)[t * S + (o & 31)] : 0.0;
            }
            cv = low && p.pad_var[pc] >= 0;
            cg.load(p.gcol + pc, npad, abase, wbase);
            pg.load(p.gpsym + pc, npad, lds_addr(L.Pv), Xbase);
            Dv = p.D[b * npad + pc];
            Ev = ri < m ? p.E[b * m + ri] : 1.0;
            if (ri < m) rg.load(p.grow + ri, m, abase, xbase);  // by ri: duplicate lanes repeat its row
            else rg.clear(abase + 8u * nnzA, xbase);
            PH(0)
        }
        // ---- run state ----
        double X = C.X[pc], DX = 0.0;
        const double Q = L.qv[pc];
        // phase-C slots: the pairs (j, w), j > w, alternate over the halves (the i-th to half
        // i & 1); the wave runs NSW(w) slots, a half without a pair there reads the zero pair
        constexpr int NS = (NB - 1 + 1) / 2;
        const int nsw = (NB - w) >> 1;  // ceil((NB - 1 - w) / 2)
        unsigned gslot[NS], tslot[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const int j = w + 1 + 2 * s + h;
            const bool v = j < NB;
            gslot[s] = lds_addr(L.gl + (v ? j * (j - 1) / 2 + w : NP) * GR * S + r);
            tslot[s] = lds_addr(L.tv + (v ? j : 0) * 16);
        }
        // the half's share of the column list (KH entries; the list is zero-padded to K)
        GatherW<KH> ch2;
#pragma unroll
        for (int k = 0; k < KH; ++k) ch2.e[k] = h ? cg.e[k + KH] : cg.e[k];
        const double r_hi = RHO_EQ_OVER_RHO_INEQ * rho;
        double y = L.ys[ri], Z = C.Z[ri], dy = 0.0;
        const signed char cl = L.ct[ri];
        const double rv = cl < 0 ? RHO_MIN : (cl > 0 ? r_hi : rho);
        const double rvi = cl < 0 ? 1.0 / RHO_MIN : (cl > 0 ? 1.0 / r_hi : 1.0 / rho);
        __syncthreads();
        if (rows_wave) L.w[ri] = rv * Z - y;  // (lanes past the padded rows may hold a stale y)
        int stop_at = p.max_iter;
        if (p.check_term) stop_at = min(stop_at, (iter / p.check_term + 1) * p.check_term);
        if (p.adaptive_rho && p.rho_interval) stop_at = min(stop_at, (iter / p.rho_interval + 1) * p.rho_interval);
        __syncthreads();
        PH(5)
        double* const cw = L.cor + w * 16;                  // c_w rows < QR
        const double* const cwh = L.cor + (h ? 128 : w * 16);  // the half's correction (upper half: zeros)
        while (iter < stop_at) {
            ++iter;
            // rhs = sigma x_prev - q + A' (rho z_prev - y), column pc: the lower half sums
            // the list's first KH entries, the upper half the rest, one permlane32 swap
            {
                double av[KH], wv[KH];
#pragma unroll
                for (int k = 0; k < KH; ++k) {
                    av[k] = lds_at(ch2.e[k] & 0xFFFFu);
                    wv[k] = lds_at(ch2.e[k] >> 16);
                }
                double v = low ? sigma * X - Q : 0.0;
#pragma unroll
                for (int k = 0; k < KH; ++k) v += av[k] * wv[k];
                const unsigned vlo = (unsigned)__double2loint(v), vhi = (unsigned)__double2hiint(v);
                const auto l2 = __builtin_amdgcn_permlane32_swap(vlo, vlo, false, false);
                const auto h2 = __builtin_amdgcn_permlane32_swap(vhi, vhi, false, false);
                const double v0 = __hiloint2double((int)h2[0], (int)l2[0]);
                const double v1 = __hiloint2double((int)h2[1], (int)l2[1]);
                if (low) L.rb[pc] = cv ? v0 + v1 : 0.0;
            }
            __syncthreads();
            PH(1)
            // A: c_w = sum_{j<w} G_wj b_j (rows rr < QR: 16 rows x 4 lanes of 8 columns), wave w only
            if (w > 0) {
                const double* gq = L.gl + (w * (w - 1) / 2) * GR * S + min(rr, GR - 1) * S + 8 * ch;
                double acc = 0.0;
#pragma unroll
                for (int j = 0; j < NB - 1; ++j) {
                    if (j < w) {
                        double bj[8], ga[8];
#pragma unroll
                        for (int e = 0; e < 8; e += 2) {
                            ld2(L.rb + j * S + 8 * ch + e, bj[e], bj[e + 1]);
                            ld2(gq + j * GR * S + e, ga[e], ga[e + 1]);
                        }
#pragma unroll
                        for (int e = 0; e < 8; ++e) acc += ga[e] * bj[e];
                    }
                }
                acc += dpp<0xB1>(acc);
                acc += dpp<0x4E>(acc);
                if (ch == 0 && rr < QR) cw[rr] = acc;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            PH(12)
            // B: t_w[r] = S_w^{-1}[r] (b_w + c_w): half-row sums, permlane32 swap
            double t;
            {
                constexpr int QE = (QR + 1) & ~1;  // c_w's nonzero rows (< amax), read in pairs
                double v[16], cc[QE];
#pragma unroll
                for (int c = 0; c < 16; c += 2) ld2(L.rb + w * S + 16 * h + c, v[c], v[c + 1]);
#pragma unroll
                for (int c = 0; c < QE; c += 2) ld2(cwh + c, cc[c], cc[c + 1]);
#pragma unroll
                for (int c = 0; c < QR; ++c) v[c] += cc[c];
                double a[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int c = 0; c < 16; ++c) a[c & 3] += SB[c] * v[c];
                const double th = (a[0] + a[1]) + (a[2] + a[3]);
                const unsigned lo = (unsigned)__double2loint(th), hi = (unsigned)__double2hiint(th);
                const auto l2 = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
                const auto h2 = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
                const double t0 = __hiloint2double((int)h2[0], (int)l2[0]);  // lower half's
                const double t1 = __hiloint2double((int)h2[1], (int)l2[1]);  // upper half's
                t = t0 + t1;
                if (low && r < QR) L.tv[w * 16 + r] = t;
            }
            __syncthreads();
            PH(13)
            // C: x~_w[r] = t + sum_s G_{pair_s}[q][r] t_{j_s}[q]  (slots split over the halves;
            // rows q < QR: the G blocks are zero from row amax on)
            {
                double a0 = 0.0, a1 = 0.0;
#pragma unroll
                for (int s = 0; s < NS; ++s) {
                    if (s < nsw) {
                        double gv[QR], tq[QR];
#pragma unroll
                        for (int q = 0; q < QR; ++q) gv[q] = lds_at(gslot[s] + q * S * 8);
#pragma unroll
                        for (int q = 0; q < QR; q += 2) lds_at2(tslot[s] + q * 8, tq[q], tq[q + 1]);
#pragma unroll
                        for (int q = 0; q < QR; q += 2) {
                            a0 += gv[q] * tq[q];
                            a1 += gv[q + 1] * tq[q + 1];
                        }
                    }
                }
                const double d = a0 + a1;
                const unsigned lo = (unsigned)__double2loint(d), hi = (unsigned)__double2hiint(d);
                const auto l2 = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
                const auto h2 = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
                const double d0 = __hiloint2double((int)h2[0], (int)l2[0]);
                const double d1 = __hiloint2double((int)h2[1], (int)l2[1]);
                const double xn = t + (d0 + d1);
                if (low) L.xt[pc] = xn;
                const double xnew = alpha * xn + (1.0 - alpha) * X;
                DX = xnew - X;
                X = xnew;
            }
            __syncthreads();
            PH(14)
            // rows: z~ = A x~ ; relaxed + projected z ; y ; next w
            if (rows_wave) {
                double av[K], xv[K];
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    av[k] = lds_at(rg.e[k] & 0xFFFFu);
                    xv[k] = lds_at(rg.e[k] >> 16);
                }
                const double lo = L.lo[ri], up = L.up[ri];
                double zt = av[0] * xv[0];
#pragma unroll
                for (int k = 1; k < K; ++k) zt += av[k] * xv[k];
                const double zr = alpha * zt + (1.0 - alpha) * Z;
                const double zn = __builtin_fmin(__builtin_fmax(zr + rvi * y, lo), up);
                const double dd = rv * (zr - zn);
                Z = zn;
                dy = dd;
                y += dd;
                L.w[ri] = rv * zn - y;
            }
            __syncthreads();
            PH(3)
        }
        // run state back to LDS
        if (low) { C.X[pc] = X; L.dx[pc] = DX; }
        if (rows_wave) { L.ys[ri] = y; C.Z[ri] = Z; C.dY[ri] = dy; }
        __syncthreads();
        can_check = p.check_term && (iter % p.check_term == 0);
        const bool do_rho = p.adaptive_rho && p.rho_interval && (iter % p.rho_interval == 0);
        if (!can_check && !do_rho) break;
        info_iter = iter;
        bool stop = false;
        {
            // inline update_info + check_termination (as solve_w2_body's), one row per thread
            const bool unscale = p.scaling && !p.scaled_term;
            const unsigned ysbase = lds_addr(L.ys), dYbase = lds_addr(C.dY), dxbase = lds_addr(L.dx);
            double mx[17], sm[2] = {0.0, 0.0}, adx = 0.0;
#pragma unroll
            for (int k = 0; k < 17; ++k) mx[k] = 0.0;
            {
                const bool ok = tid < m;
                double ax = 0.0, ad = 0.0;
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const unsigned e = rg.e[k], va = e >> 16;
                    const double a = lds_at(e & 0xFFFFu);
                    ax += a * lds_at(va - xbase + Xbase);
                    ad += a * lds_at(va - xbase + dxbase);
                }
                adx = ad;
                const double zi = Z, pr = ax - zi, ei = 1.0 / Ev;
                const double lo = L.lo[ri], up = L.up[ri];
                double d = dy;
                if (up > OSQP_INFTY * MIN_SCALING) d = (lo < -OSQP_INFTY * MIN_SCALING) ? 0.0 : cmin(d, 0.0);
                else if (lo < -OSQP_INFTY * MIN_SCALING) d = cmax(d, 0.0);
                if (ok) {
                    mx[0] = fabs(ei * pr);
                    mx[2] = fabs(ei * zi);
                    mx[3] = fabs(ei * ax);
                    mx[7] = fabs(pr);
                    mx[9] = fabs(zi);
                    mx[10] = fabs(ax);
                    mx[14] = fabs(unscale ? Ev * d : d);
                    sm[0] = up * cmax(d, 0.0) + lo * cmin(d, 0.0);
                    C.dY[ri] = d;
                }
            }
            {  // the lane's column (lower half): P x, A' y, P dx, and the delta x norm
                double px = 0.0, pdx = 0.0, aty = 0.0;
#pragma unroll
                for (int k = 0; k < KPK; ++k) {
                    const unsigned e = pg.e[k], va = e >> 16;
                    const double pv = lds_at(e & 0xFFFFu);
                    px += pv * lds_at(va);
                    pdx += pv * lds_at(va - Xbase + dxbase);
                }
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const unsigned e = cg.e[k];
                    aty += lds_at(e & 0xFFFFu) * lds_at((e >> 16) - wbase + ysbase);
                }
                if (cv) {
                    const double d = (Q + px) + aty, di = 1.0 / Dv;
                    mx[1] = fabs(di * d);
                    mx[4] = fabs(di * Q);
                    mx[5] = fabs(di * aty);
                    mx[6] = fabs(di * px);
                    mx[8] = fabs(d);
                    mx[11] = fabs(Q);
                    mx[12] = fabs(aty);
                    mx[13] = fabs(px);
                    mx[15] = fabs(unscale ? Dv * DX : DX);
                    mx[16] = fabs(unscale ? pdx * di : pdx);
                }
            }
            if (tid < npad && p.pad_var[tid] >= 0) sm[1] = L.qv[tid] * L.dx[tid];
            block_max_sum_tr<T8, 17, 2>(mx, sm, red8);
            Res R;
            if (unscale) {
                R.pri = mx[0]; R.dua = cinv * mx[1];
                R.nz = mx[2]; R.nax = mx[3]; R.nq = mx[4]; R.naty = mx[5]; R.npx = mx[6];
            } else {
                R.pri = mx[7]; R.dua = mx[8];
                R.nz = mx[9]; R.nax = mx[10]; R.nq = mx[11]; R.naty = mx[12]; R.npx = mx[13];
            }
            R.rpri = mx[7]; R.rdua = mx[8]; R.rz = mx[9]; R.rax = mx[10]; R.rq = mx[11]; R.raty = mx[12]; R.rpx = mx[13];
            if (m == 0) R.pri = 0.0;
            if (tid == 0) R.save(L.res);
            if (can_check) {
                int st = MPCQP_UNSOLVED_;
                double obj = 0.0;
                bool done = false;
                if (R.pri > OSQP_INFTY || R.dua > OSQP_INFTY) {
                    st = MPCQP_NON_CVX_;
                    obj = __builtin_nan("");
                    done = true;
                } else {
                    const bool prim_ok = m == 0 || R.pri < p.eps_abs + p.eps_rel * cmax(R.nz, R.nax);
                    double mxd = cmax(cmax(R.nq, R.naty), R.npx);
                    if (unscale) mxd *= cinv;
                    const bool dual_ok = R.dua < p.eps_abs + p.eps_rel * mxd;
                    bool prim_inf = false, dual_inf = false;
                    if (!prim_ok || !dual_ok) {
                        const double norm_dy = mx[14], norm_dx = mx[15], epi = p.eps_pinf, edi = p.eps_dinf;
                        const double cs = unscale ? cval : 1.0;
                        if (!prim_ok && m != 0 && norm_dy > epi && sm[0] < epi * norm_dy) {
                            __syncthreads();
                            double na[1] = {0.0};
                            double a = 0.0;
#pragma unroll
                            for (int k = 0; k < K; ++k) {
                                const unsigned e = cg.e[k];
                                a += lds_at(e & 0xFFFFu) * lds_at((e >> 16) - wbase + dYbase);
                            }
                            if (cv) na[0] = fabs(unscale ? a * (1.0 / Dv) : a);
                            block_max<T8, 1>(na, L.red);
                            prim_inf = na[0] < epi * norm_dy;
                        }
                        if (!dual_ok && norm_dx > edi && sm[1] < cs * edi * norm_dx && mx[16] < cs * edi * norm_dx) {
                            bool viol = false;
                            if (tid < m) {
                                const double ar = unscale ? adx * (1.0 / Ev) : adx;
                                const double lo = L.lo[ri], up = L.up[ri];
                                if ((up < OSQP_INFTY * MIN_SCALING && ar > edi * norm_dx) ||
                                    (lo > -OSQP_INFTY * MIN_SCALING && ar < -edi * norm_dx))
                                    viol = true;
                            }
                            dual_inf = !block_any<T8>(viol, L.flag);
                        }
                    }
                    if (prim_ok && dual_ok) {
                        st = MPCQP_SOLVED_;
                        done = true;
                    } else if (prim_inf) {
                        st = MPCQP_PRIMAL_INFEASIBLE_;
                        obj = OSQP_INFTY;
                        if (tid == 0) L.flag[3] = unscale;
                        done = true;
                    } else if (dual_inf) {
                        st = MPCQP_DUAL_INFEASIBLE_;
                        obj = -OSQP_INFTY;
                        if (tid == 0) L.flag[2] = unscale;
                        done = true;
                    }
                }
                __syncthreads();
                if (done && tid == 0) { L.flag[1] = st; L.res[14] = obj; }
                __syncthreads();
                status = done ? st : MPCQP_UNSOLVED_;
                stop = done;
            }
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
        update_info_nl<T8>(p.self, b, cinv);
        info_iter = iter;
        status = check_termination_nl<T8>(p.self, b, cval, cinv, 0);
    }
    const bool has_sol = !(status == MPCQP_PRIMAL_INFEASIBLE_ || status == MPCQP_PRIMAL_INFEASIBLE_INACCURATE_ ||
                           status == MPCQP_DUAL_INFEASIBLE_ || status == MPCQP_DUAL_INFEASIBLE_INACCURATE_ ||
                           status == MPCQP_NON_CVX_);
    if (has_sol) objective_nl<T8>(p.self, cinv);
    if (status == MPCQP_UNSOLVED_) {
        status = check_termination_nl<T8>(p.self, b, cval, cinv, 1);
        if (status == MPCQP_UNSOLVED_) status = MPCQP_MAX_ITER_REACHED_;
    }
    finalize_nl<T8>(p.self, b, xo, yo, cinv, rho, status, info_iter, rho_updates, p.ostat, p.oiter);
#ifdef MPCQP_PHASE_PROF
    if (prof) {
        __syncthreads();
        PH(5)
        if (tid == 0) {
#pragma unroll
            for (int k = 0; k < 6; ++k) p.prof[b * kProfSlots + k] = L.pacc[k];
#pragma unroll
            for (int k = 8; k < 15; ++k) p.prof[b * kProfSlots + k] = L.pacc[k];
            p.prof[b * kProfSlots + 2] = L.pacc[12] + L.pacc[13] + L.pacc[14];
            p.prof[b * kProfSlots + 6] = clock64() - t0c;
            p.prof[b * kProfSlots + 7] = wall_clock64() - t0w;
            p.prof[b * kProfSlots + 15] = t0w;
        }
    }
#endif
#undef PH
}

template <int K, int KPK>
__global__ __launch_bounds__(T8, 1) void k_solve_w8(KParams p, double* __restrict__ xo, double* __restrict__ yo,
                                                    int factor_only) {
    solve_w8_body<K, KPK>(p, xo, yo, factor_only);
    extern __shared__ __attribute__((aligned(16))) double sm[];
    order_epilogue<T8>(p, (int*)sm);
}

#endif  // MPCQP_EXPERIMENTAL

// Host-side guard tying an instantiation's compile-time list lengths to the plan: gather
// lists are kGS deep in memory (plan.cpp), so a shorter K never reads out of the list, but
// it would drop A entries; K / KC: row / column gather lengths, KPK: P terms per column,
// QR: nonzero G rows, K1: the slot-1 rows' length (two-wave kernel)
static hipError_t lists_fit(const KParams& p, int K, int KC, int KPK, int QR, int K1 = 1 << 30) {
    const bool ok = p.gkr <= K && p.gkc <= KC && p.gk <= std::max(K, KC) && p.pk <= KPK && p.amax <= QR &&
                    p.gk1 <= K1 && K <= kGS && KC <= kGS;
    return ok ? hipSuccess : hipErrorInvalidValue;
}

// the four-wave kernel's dense-inverse form (DK) for plans without eliminated columns whose
// blocks have at most NB0 = 26 (blocks 0, 1) / NB1 = 28 (blocks 2, 3) real columns
// (plan.cpp balances the four blocks for it): measured and not taken, so it is
// compiled into the experimental builds only, where MPCQP_DENSE_W4=1 turns it on (and the
// planner's balanced merge with it)
bool dense_w4_on() {
#ifdef MPCQP_EXPERIMENTAL
    static const bool on = [] {
        const char* e = getenv("MPCQP_DENSE_W4");
        return e && e[0] == '1';
    }();
    return on;
#else
    return false;
#endif
}
[[maybe_unused]] static bool dense_w4(const KParams& p) {
    return dense_w4_on() && p.ne == 0 && p.Kd && p.bsz01 <= 26 && p.bsz23 <= 28;
}

// the fused kernel's instantiation for the plan, or 0: variant 10 and the 128-thread
// register-list setup shape (one padded column per thread, two rows, four A values)
static int setup_solve_fits(const KParams& p) {
    if (p.variant == 17) return p.pk <= 4;  // variant_fits(17) covers the rest (list lengths, nnzA <= 2 or 3 x T4)
    return p.variant == 10 && p.npad <= T2 && p.m <= 2 * T2 && p.gk <= 6 && p.pk <= 4 && p.nnzA <= 4 * T2 &&
           p.nnzP <= 2 * T2;
}

int one_shot_form(const KParams& p, size_t* lds) {
    if (p.variant != 17 || p.polish || !setup_solve_fits(p)) return 0;
    const size_t base = std::max(lds_w2_bytes(p), lds_setup_r_bytes(p.nnzP, p.nnzA, p.npad, p.m));
    // (form 2: the G blocks and the y of a refactorisation, which the factorisation's E tiles
    // overwrite in the carve, after the S_k^{-1} tiles)
    const size_t g = sizeof(double) * ((size_t)(p.nb * (p.nb - 1) / 2) * p.amax * S + (size_t)p.m);
    // form 3 (GL 2): the G blocks straight into the solve's gl copy, with factorize_w4_gl's
    // scratch (the E tiles and wave buffers) in the carve's V span before gl
    // form 2 also keeps E and D after gl (edl_E / edl_D: the V span's room past gl)
    const long vspan = 3L * solve_mpad(p.m) + 2L * p.npad;
    const long vfree = solve_vlen(p.m, p.npad, p.nb, p.amax, p.mode) - vspan - solve_glen(p.nb, p.amax, p.mode);
    const bool edl = vfree >= ((p.m + 1) & ~1) + p.npad;
    const int form = base + g <= 80 * 1024 && edl ? 2 : (p.amax <= 8 && 4L * p.amax * S + 8 * S + 8 <= vspan ? 3 : 1);
    if (lds) *lds = form == 2 ? base + g : base;
    return form;
}

hipError_t launch_setup_solve(const KParams& p, long B, const double* Px, const double* Ax, const double* q,
                              const double* l, const double* u, double* xo, double* yo, hipStream_t st,
                              bool one_shot) {
    size_t lds1 = 0;
    const int form = one_shot ? one_shot_form(p, &lds1) : 0;
    if (form) {
        decltype(&k_setup_solve_w4<6, 4, 5, 6, 2>) k4;
        if (form == 2)
            k4 = p.ne ? k_setup_solve_w4<6, 4, 8, 8, 3, true, 8, false, true, 1>
                      : (p.amax <= 5 ? k_setup_solve_w4<6, 4, 5, 6, 2, false, 6, false, true, 1>
                                     : k_setup_solve_w4<6, 4, 8, 6, 2, false, 6, false, true, 1>);
        else if (form == 3)
            k4 = p.ne ? k_setup_solve_w4<6, 4, 8, 8, 3, true, 8, false, true, 2>
                      : (p.amax <= 5 ? k_setup_solve_w4<6, 4, 5, 6, 2, false, 6, false, true, 2>
                                     : k_setup_solve_w4<6, 4, 8, 6, 2, false, 6, false, true, 2>);
        else
            k4 = p.ne ? k_setup_solve_w4<6, 4, 8, 8, 3, true, 8, false, true>
                      : (p.amax <= 5 ? k_setup_solve_w4<6, 4, 5, 6, 2, false, 6, false, true>
                                     : k_setup_solve_w4<6, 4, 8, 6, 2, false, 6, false, true>);
        hipError_t e = lists_fit(p, 6, p.ne ? 8 : 6, 4, p.ne || p.amax > 5 ? 8 : 5);
        if (e != hipSuccess) return e;
        e = hipFuncSetAttribute((const void*)k4, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds1);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k4, dim3((unsigned)B), dim3(T4), lds1, st, p, Px, Ax, q, l, u, xo, yo);
        return hipGetLastError();
    }
#ifdef MPCQP_EXPERIMENTAL
    if (p.variant == 19) {
        hipError_t e = launch_setup_solve_heavy(p, B, Px, Ax, q, l, u, xo, yo, st);
        return (e != hipSuccess || !p.polish) ? e : launch_polish(p, B, xo, yo, st);
    }
#endif
    if (!setup_solve_fits(p)) {
        hipError_t e = launch_setup(p, B, Px, Ax, q, l, u, st);
        return e != hipSuccess ? e : launch_solve(p, B, xo, yo, 0, st);
    }
    const size_t lds = std::max(lds_w2_bytes(p), lds_setup_r_bytes(p.nnzP, p.nnzA, p.npad, p.m));
    if (p.variant == 17) {
        // QR: rows of the G blocks phase C sums (the nonzero ones: amax)
        // EL (eliminated columns, the slack layouts): three A values per setup thread
        auto k4 = p.ne ? k_setup_solve_w4<6, 4, 8, 8, 3, true, 8>
                       : (p.amax <= 5 ? k_setup_solve_w4<6, 4, 5, 6, 2> : k_setup_solve_w4<6, 4, 8, 6, 2>);
#ifdef MPCQP_EXPERIMENTAL
        if (!p.ne && p.amax <= 5 && dense_w4(p)) k4 = k_setup_solve_w4<6, 4, 5, 6, 2, false, 6, true>;
#endif
        hipError_t e = lists_fit(p, 6, p.ne ? 8 : 6, 4, p.ne || p.amax > 5 ? 8 : 5);
        if (e != hipSuccess) return e;
        e = hipFuncSetAttribute((const void*)k4, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k4, dim3((unsigned)B), dim3(T4), lds, st, p, Px, Ax, q, l, u, xo, yo);
        e = hipGetLastError();
        if (e != hipSuccess || !p.polish) return e;
        return launch_polish(p, B, xo, yo, st);
    }
    auto k = p.gk1 <= 1 ? k_setup_solve_w2<6, 2, 4, 1, 6, 2, 4, 2> : k_setup_solve_w2<6, 2, 4, 6, 6, 2, 4, 2>;
    hipError_t e = lists_fit(p, 6, 6, 4, 1 << 30, 6);
    if (e != hipSuccess) return e;
    e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3((unsigned)B), dim3(T2), lds, st, p, Px, Ax, q, l, u, xo, yo);
    e = hipGetLastError();
    if (e != hipSuccess || !p.polish) return e;
    return launch_polish(p, B, xo, yo, st);
}

template <int K, int RS, int KPK, int K1>
static hipError_t go_w2(const KParams& p, long B, double* xo, double* yo, int fo, hipStream_t st, size_t lds,
                        KernelRef* ref) {
    auto k = k_solve_w2<K, RS, KPK, K1>;
    hipError_t e = lists_fit(p, K, K, KPK, 1 << 30, K1);
    if (e != hipSuccess) return e;
    if (ref) { *ref = {(const void*)k, T2, lds}; return hipSuccess; }
    e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3((unsigned)B), dim3(T2), lds, st, p, xo, yo, fo);
    return hipGetLastError();
}

#ifdef MPCQP_EXPERIMENTAL
template <int K, int RS>
static hipError_t go_w(const KParams& p, long B, double* xo, double* yo, int fo, hipStream_t st, size_t lds,
                       KernelRef* ref) {
    auto k = k_solve_w<K, RS>;
    if (ref) { *ref = {(const void*)k, TW, lds}; return hipSuccess; }
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3((unsigned)B), dim3(TW), lds, st, p, xo, yo, fo);
    return hipGetLastError();
}
#endif

// the two-wave kernel's LDS: the carve plus the nb S_k^{-1} tiles
size_t lds_w2_bytes(const KParams& p) {
    return 16 * ((lds_base_bytes(p) + 15) / 16) + sizeof(double) * (size_t)p.nb * SS;
}

// Wave-kernel instantiations (solve.hip::variant_fits gives their preconditions).
hipError_t launch_solve_wave(const KParams& p, long B, double* xo, double* yo, int factor_only, hipStream_t st,
                             KernelRef* ref) {
    [[maybe_unused]] const size_t lds = lds_solve_bytes(p);  // (the experimental variants')
    switch (p.variant) {
#ifdef MPCQP_EXPERIMENTAL
        case 8: return go_w<6, 3>(p, B, xo, yo, factor_only, st, lds, ref);
        case 9: return go_w<8, 4>(p, B, xo, yo, factor_only, st, lds, ref);
#endif
        case 17: {
            auto k = factor_only
                         ? (p.ne ? k_solve_w4<6, 4, 8, true, 8, true>
                                 : (p.amax <= 5 ? k_solve_w4<6, 4, 5, false, 6, true> : k_solve_w4<6, 4, 8, false, 6, true>))
                         : (p.ne ? k_solve_w4<6, 4, 8, true, 8>
                                 : (p.amax <= 5 ? k_solve_w4<6, 4, 5> : k_solve_w4<6, 4, 8>));
#ifdef MPCQP_EXPERIMENTAL
            if (!factor_only && !p.ne && p.amax <= 5 && dense_w4(p)) k = k_solve_w4<6, 4, 5, false, 6, false, true>;
#endif
            const size_t lds = lds_w2_bytes(p);
            hipError_t e = lists_fit(p, 6, p.ne ? 8 : 6, 4, p.ne || p.amax > 5 ? 8 : 5);
            if (e != hipSuccess) return e;
            if (ref) { *ref = {(const void*)k, T4, lds}; return hipSuccess; }
            e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL(k, dim3((unsigned)B), dim3(T4), lds, st, p, xo, yo, factor_only);
            return hipGetLastError();
        }
#ifdef MPCQP_EXPERIMENTAL
        case 18: {
            auto k = k_solve_w8<8, 8>;
            if (ref) { *ref = {(const void*)k, T8, lds}; return hipSuccess; }
            hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL(k, dim3((unsigned)B), dim3(T8), lds, st, p, xo, yo, factor_only);
            return hipGetLastError();
        }
#endif
        case 10:  // slot-1 rows (>= 128) with at most one nonzero (cfg 2's box rows): K1 = 1
            return p.gk1 <= 1 ? go_w2<6, 2, 4, 1>(p, B, xo, yo, factor_only, st, lds_w2_bytes(p), ref)
                              : go_w2<6, 2, 4, 6>(p, B, xo, yo, factor_only, st, lds_w2_bytes(p), ref);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace mpcqp
