// solve_dense.hip -- the ADMM kernel for small QPs (n <= R variables) with the
// reduced KKT matrix inverted explicitly: M^{-1}, M = P + sigma I + A' diag(rho) A,
// one dense row per lane pair in registers.
//
// Why: the block-tridiagonal solve of solve_wave.hip (k_solve_w2) runs the
// x-update as three dependent phases (L^{-1}, S^{-1}, L^{-T}) with an LDS round
// trip and a (wave) barrier between each; at cfg 2 (n = 104) they cost ~2,200 of
// the ~3,400 cycles of an iteration, nearly all of it latency.  With the inverse
// in registers the x-update is one phase: every lane reads half of the rhs as
// 16-byte LDS broadcasts and does R/2 fp64 FMAs for its half row, and the lane
// pair adds its halves with one DPP swap.  An iteration is then
//   rhs   b_j = sigma x_j - q_j + A'(rho z - y)_j   (lane (j,0), column gather) -> bc (LDS)
//   solve x~_j = sum_k Minv[j][k] b_k               (lanes (j,0), (j,1))       -> xt (LDS)
//   rows  z~ = A x~, relaxation, projection, y update, w = rho z - y          -> w  (LDS)
// with three workgroup barriers and no wave barriers.  Lane t = 2 j + h holds
// columns [h R/2, h R/2 + R/2) of row j: R/2 doubles, so the rows of the 104 x 104
// inverse of cfg 2 take 104 VGPRs and the kernel runs two waves per SIMD (two QPs
// per CU, as the block kernel): a whole row per lane (208 VGPRs) left too few
// registers for the LDS reads in flight.
//
// The inverse: M is assembled row by row through an LDS staging area (chunks of
// rows; the staging aliases the per-iteration vectors, as the block factorisation's
// scratch does) and inverted in place by Gauss-Jordan on the register rows.
// Variables are in their natural order 0..n-1 (lane j owns variable j); rows
// n..R-1 are identity rows, so the in-place inverse stays a static R x R loop.
// The pivot loop is rolled: after pivot p every lane shifts its half row by one
// (the shift is the FMA's destination; the element that crosses from the second
// half into the first comes over with the same DPP swap that brings M[j][p] to the
// second lane), so the pivot column is always element 0 of the first half and
// after R pivots the row is back in natural order.  Pivot row p is
// published through LDS by the lanes that hold column p (M_pj = +-M_jp, the
// in-place Gauss-Jordan matrix of a symmetric input being symmetric up to sign),
// one double per lane, double-buffered so one barrier per pivot suffices.
// A non-positive pivot means M is not positive definite: OSQP's "non convex".
//
// Everything else -- data loads, warm start, the inline termination check,
// adaptive rho, the out-of-line objective / final check / store -- follows
// k_solve_w2 (OSQP 0.6 osqp_solve behind vehicle_lateral_mpc_slack_increment.py:248
// and Control/MPC/mpc_kinematics.py:196; oracle/osqp_oracle.c restates it).
#include <hip/hip_runtime.h>

#include "solve_phases.h"
#include "wave_util.h"

namespace mpcqp {

constexpr int TD = 256;

// d = a * b + c as a VOP3 v_fma_f64 with its own destination: the compiler's
// two-address form (v_fmac_f64) would add a v_mov per element of the row shift
__device__ __forceinline__ double fma3(double a, double b, double c) {
    double d;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

// LDS beyond the base carve (solve_phases.h::carve): bc[R] (compact rhs), v2p[R] (int),
// two pivot buffers of two parity copies of 2R + 2 doubles
__host__ __device__ inline long dense_extra_doubles(int R) { return 2L * R + 2L * 2 * (2L * R + 2) + 4; }

template <int R, int K, int RS, int KPK>
__global__ __launch_bounds__(TD, 2) void k_solve_d(KParams p, double* __restrict__ xo, double* __restrict__ yo,
                                                   int factor_only) {
    static_assert(R % 4 == 0, "half rows must be whole 16-byte pairs");
    constexpr int H = R / 2;
    const int tid = threadIdx.x, jr = tid >> 1, h = tid & 1;  // row jr, half h
    const long b = instance_of(p);
    const int n = p.n, m = p.m, npad = p.npad, nnzP = p.nnzP, nnzA = p.nnzA;
    SL2 C = carve(p);
    SLds& L = C.L;
    extern __shared__ __attribute__((aligned(16))) double smd[];
    double* const bc = A16(smd + (lds_base_bytes(p) + 15) / 16 * 2);
    int* const v2p = (int*)(bc + R);
    double* const pbuf = A16(bc + R + (R + 1) / 2 + 1);  // [2 buffers][2 parities][2R + 2]
    constexpr int PBL = 2 * R + 2;

    if (p.err[b]) {  // invalid data (flagged by setup/update): NaN outputs
        for (int j = tid; j < n; j += TD) if (xo) xo[b * n + j] = __builtin_nan("");
        for (int i = tid; i < m; i += TD) if (yo) yo[b * m + i] = __builtin_nan("");
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
    for (int e = tid; e < nnzA; e += TD) L.Acsc[e] = p.Ax[b * nnzA + e];
    if (tid == 0) L.Acsc[nnzA] = 0.0;  // the gather lists' padding slot
    for (int v = tid; v < nnzP; v += TD) L.Pv[v] = p.Px[b * nnzP + v];
    if (tid == 0) L.Pv[nnzP] = 0.0;
    const int mp = solve_mpad(m);
    for (int i = tid; i < mp; i += TD) {  // rows >= m: inert padding (l = u = 0, z = 0)
        const bool in = i < m;
        L.lo[i] = in ? p.l[b * m + i] : 0.0;
        L.up[i] = in ? p.u[b * m + i] : 0.0;
        L.ct[i] = in ? p.ct[b * m + i] : 0;
        C.Z[i] = (in && warm) ? p.z[b * m + i] : 0.0;
    }
    for (int pc = tid; pc < npad; pc += TD) {
        L.qv[pc] = p.q[b * npad + pc];
        C.X[pc] = warm ? p.x[b * npad + pc] : 0.0;
        const int j = p.pad_var[pc];
        if (j >= 0) v2p[j] = pc;
    }
    for (int j = n + tid; j < R; j += TD) v2p[j] = -1;  // (v2p of rows >= n is never read)
    for (int j = tid; j < R; j += TD) bc[j] = 0.0;  // rows n..R-1 of the rhs stay zero
    if (tid < 16) L.res[tid] = 0.0;
    if (tid < 4) L.flag[tid] = 0;
    __syncthreads();
    const int pcs = jr < n ? v2p[jr] : 0;  // the row's variable, as a padded column
    const bool cv = h == 0 && jr < n;        // the lane that owns variable jr

    int status = MPCQP_UNSOLVED_, rho_updates = 0, iter = 0, info_iter = 0;
    bool can_check = false, need_factor = true;
    double Mr[H];  // row jr of M^{-1}, columns [h H, h H + H) (rows >= R: unused)
#pragma unroll
    for (int j = 0; j < H; ++j) Mr[j] = 0.0;
    PH(5)
    for (;;) {
        __syncthreads();
        if (need_factor) {  // start, and after a rho change
            need_factor = false;
            // the staging area aliases ys (and w, rb, xt, dY): y waits in the workspace
            if (iter > 0)
                for (int i = tid; i < m; i += TD) p.y[b * m + i] = L.ys[i];
            __syncthreads();
            // ---- assemble M = P + sigma I + A' diag(rho) A, RC rows at a time ----
            double* const ST = L.SP;
            const int RC = min(R, (int)(3 * SS / R));
#pragma unroll 1
            for (int c0 = 0; c0 < R; c0 += RC) {
                for (int o = tid; o < RC * R; o += TD) ST[o] = 0.0;
                __syncthreads();
                const bool mine = jr >= c0 && jr < c0 + RC && jr < R;
                if (mine && h == 0) {
                    double* row = ST + (jr - c0) * R;
                    if (cv) {
                        row[jr] += sigma;
                        const int* pl = p.gpsym + pcs;
#pragma unroll 1
                        for (int k = 0; k < p.pk; ++k) {
                            const unsigned e = (unsigned)pl[(long)k * npad];
                            const int idx = (int)(e & 0xFFFFu), j = p.pad_var[e >> 16];
                            if (idx < nnzP && j >= 0) row[j] += L.Pv[idx];
                        }
                        const int* cl = p.gcol + pcs;
#pragma unroll 1
                        for (int k = 0; k < p.gk; ++k) {
                            const unsigned e = (unsigned)cl[(long)k * npad];
                            const int a = (int)(e & 0xFFFFu), i = (int)(e >> 16);
                            if (a >= nnzA) continue;
                            const double wa = rho_of(L.ct[i], rho) * L.Acsc[a];
                            const int* rl = p.grow + i;
#pragma unroll 1
                            for (int k2 = 0; k2 < p.gk; ++k2) {
                                const unsigned e2 = (unsigned)rl[(long)k2 * m];
                                const int a2 = (int)(e2 & 0xFFFFu), j = p.pad_var[e2 >> 16];
                                if (a2 < nnzA && j >= 0) row[j] += wa * L.Acsc[a2];
                            }
                        }
                    } else {
                        row[jr] = 1.0;  // rows n..R-1: identity
                    }
                }
                __syncthreads();
                if (mine) {
                    const double* row = ST + (jr - c0) * R + h * H;
#pragma unroll
                    for (int j = 0; j < H; j += 2) ld2(row + j, Mr[j], Mr[j + 1]);
                }
                __syncthreads();
            }
            PH(8)
            // ---- Gauss-Jordan inverse in place, rolled pivot loop with a row shift ----
            double minpiv = 1.0;  // -1 once a pivot is not positive (NaN-safe)
#pragma unroll 1
            for (int pv = 0; pv < R; ++pv) {
                double* const A0 = pbuf + (pv & 1) * 2 * PBL;  // parity-0 copy: A0[c] = A0[c + R] = v_c
                double* const A1 = A0 + PBL;                   // parity-1 copy: A1[c + 1] = A1[c + 1 + R] = v_c
                const double sw = dpp<0xB1>(Mr[0]);            // the partner lane's element 0
                const double a = h ? sw : Mr[0];               // M[jr][pv]
                if (h == 0 && jr < R) {
                    const double v = jr < pv ? -a : a;         // row pv = +-column pv
                    A0[jr] = v;
                    A0[jr + R] = v;
                    A1[jr + 1] = v;
                    A1[jr + 1 + R] = v;
                }
                __syncthreads();
                // pivot row, rotated: prow[k] = v_{pv+k}; the lane reads prow[1 + h H + j], j < H,
                // from whichever copy puts that run on a 16-byte boundary
                const double piv = A0[pv];
                const double* nx = A16(((pv & 1) ? A0 + pv + 1 : A1 + pv + 2) + h * H);
                minpiv = piv > 0.0 ? minpiv : -1.0;
                double d = __builtin_amdgcn_rcp(piv);
                d = __builtin_fma(d, __builtin_fma(-piv, d, 1.0), d);
                d = __builtin_fma(d, __builtin_fma(-piv, d, 1.0), d);
                // the row update, in batches of GB pairs of pivot-row values (all LDS reads of a
                // batch in flight before the first use)
                constexpr int GB = 8;
                const bool prow_lane = jr == pv;  // the pivot row: row / piv, and 1 / piv in the new column
                const double nc = -(a * d);
#pragma unroll
                for (int j0 = 0; j0 < H; j0 += 2 * GB) {
                    double u[2 * GB];
#pragma unroll
                    for (int q = 0; q < 2 * GB; q += 2)
                        if (j0 + q < H) ld2(nx + j0 + q, u[q], u[q + 1]);
                    if (prow_lane) {
#pragma unroll
                        for (int q = 0; q < 2 * GB; ++q)
                            if (j0 + q < H) Mr[j0 + q] = u[q] * d;
                    } else {
#pragma unroll
                        for (int q = 0; q < 2 * GB; ++q) {
                            const int j = j0 + q;
                            if (j < H - 1) Mr[j] = fma3(nc, u[q], Mr[j + 1]);
                            else if (j == H - 1) Mr[j] = h ? nc : fma3(nc, u[q], sw);
                        }
                    }
                }
                if (prow_lane && h) Mr[H - 1] = d;
            }
            if (tid < 64) L.flag[0] = 0;
            __syncthreads();
            if (jr < R && !(minpiv > 0.0)) L.flag[0] = 1;
            __syncthreads();
            const bool ok = L.flag[0] == 0;
            __syncthreads();
            PH(10)
            if (!ok) {
                if (iter == 0) {
                    for (int j = tid; j < n; j += TD) if (xo) xo[b * n + j] = __builtin_nan("");
                    for (int i = tid; i < m; i += TD) if (yo) yo[b * m + i] = __builtin_nan("");
                    if (tid == 0) fail_status(p, b);
                    return;
                }
                status = MPCQP_NON_CVX_;
                can_check = true;  // skip the final check_termination
                break;
            }
            if (factor_only) return;
            const bool have_y = iter > 0 || warm;
            for (int i = tid; i < mp; i += TD) L.ys[i] = (have_y && i < m) ? p.y[b * m + i] : 0.0;
            __syncthreads();
            PH(0)
        }
        // ---- run state ----
        double X = cv ? C.X[pcs] : 0.0, DX = 0.0;
        const double Q = cv ? L.qv[pcs] : 0.0;
        const unsigned abase = lds_addr(L.Acsc), wbase = lds_addr(L.w), xbase = lds_addr(L.xt);
        const unsigned Xbase = lds_addr(C.X);
        GatherW<K> cg;
        if (cv) cg.load(p.gcol + pcs, npad, abase, wbase);
        else cg.clear(abase + 8u * nnzA, wbase);
        GatherW<K> rg[RS];
        double y[RS], Z[RS], dy[RS], rv[RS], rvi[RS];
        int ri[RS];
        const double r_hi = RHO_EQ_OVER_RHO_INEQ * rho;
#pragma unroll
        for (int s = 0; s < RS; ++s) {
            const int i = min(tid + s * TD, mp - 1);  // lanes past the padded rows repeat the inert last row
            ri[s] = i;
            dy[s] = 0.0;
            if (i < m) rg[s].load(p.grow + i, m, abase, xbase);
            else rg[s].clear(abase + 8u * nnzA, xbase);
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
        while (iter < stop_at) {
            ++iter;
            // rhs = sigma x_prev - q + A' (rho z_prev - y), own variable
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
                if (cv) bc[jr] = v;
            }
            __syncthreads();
            PH(1)
            // x~ = M^{-1} b: the lane's half row against the broadcast rhs, pair sum by DPP
            {
                double acc[4] = {0.0, 0.0, 0.0, 0.0};
                const double* bh = A16(bc + h * H);
                constexpr int MB = 26;  // rhs values per batch of LDS reads
#pragma unroll
                for (int j0 = 0; j0 < H; j0 += MB) {
                    double bv[MB];
#pragma unroll
                    for (int q = 0; q < MB; q += 2)
                        if (j0 + q < H) ld2(bh + j0 + q, bv[q], bv[q + 1]);
#pragma unroll
                    for (int q = 0; q < MB; ++q)
                        if (j0 + q < H) acc[q & 3] = __builtin_fma(Mr[j0 + q], bv[q], acc[q & 3]);
                }
                const double part = (acc[0] + acc[1]) + (acc[2] + acc[3]);
                const double xn = part + dpp<0xB1>(part);
                if (cv) L.xt[pcs] = xn;
                const double xnew = alpha * xn + (1.0 - alpha) * X;
                DX = xnew - X;
                X = xnew;
            }
            __syncthreads();
            PH(2)
            // z~ = A x~ ; relaxed + projected z ; y ; next w
            {
                double av[RS][K], xv[RS][K], lo[RS], up[RS];
#pragma unroll
                for (int s = 0; s < RS; ++s) {
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        av[s][k] = lds_at(rg[s].e[k] & 0xFFFFu);
                        xv[s][k] = lds_at(rg[s].e[k] >> 16);
                    }
                    lo[s] = L.lo[ri[s]];
                    up[s] = L.up[ri[s]];
                }
#pragma unroll
                for (int s = 0; s < RS; ++s) {
                    double zt = av[s][0] * xv[s][0];
#pragma unroll
                    for (int k = 1; k < K; ++k) zt += av[s][k] * xv[s][k];
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
        // run state back to LDS for the checks
        if (cv) {
            C.X[pcs] = X;
            L.dx[pcs] = DX;
        }
#pragma unroll
        for (int s = 0; s < RS; ++s) { L.ys[ri[s]] = y[s]; C.Z[ri[s]] = Z[s]; C.dY[ri[s]] = dy[s]; }
        __syncthreads();
        can_check = p.check_term && (iter % p.check_term == 0);
        const bool do_rho = p.adaptive_rho && p.rho_interval && (iter % p.rho_interval == 0);
        if (!can_check && !do_rho) break;  // max_iter reached
        info_iter = iter;
        bool stop = false;
        {
            // ---- inline update_info + check_termination: as k_solve_w2 (solve_wave.hip),
            // with the lane's own variable as its column ----
            const bool unscale = p.scaling && !p.scaled_term;
            const unsigned ysbase = lds_addr(L.ys), dYbase = lds_addr(C.dY), dxbase = lds_addr(L.dx);
            // (the scalings and the P list are only needed here: loaded per check)
            GatherW<KPK> pg;
            if (cv) pg.load(p.gpsym + pcs, npad, lds_addr(L.Pv), Xbase);
            else pg.clear(lds_addr(L.Pv) + 8u * nnzP, Xbase);
            const double Dv = cv ? p.D[b * npad + pcs] : 1.0;
            double Ev[RS];
#pragma unroll
            for (int s = 0; s < RS; ++s) Ev[s] = ri[s] < m ? p.E[b * m + ri[s]] : 1.0;
            double mx[17], sm[2] = {0.0, 0.0}, adx[RS];
#pragma unroll
            for (int k = 0; k < 17; ++k) mx[k] = 0.0;
#pragma unroll
            for (int s = 0; s < RS; ++s) {  // rows: A x, z, the projected delta y, A dx
                const bool ok = tid + s * TD < m;
                double ax = 0.0, ad = 0.0;
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const unsigned e = rg[s].e[k], va = e >> 16;
                    const double a = lds_at(e & 0xFFFFu);
                    ax += a * lds_at(va - xbase + Xbase);
                    ad += a * lds_at(va - xbase + dxbase);
                }
                adx[s] = ad;
                const double zi = Z[s], pr = ax - zi, ei = 1.0 / Ev[s];
                const double lo = L.lo[ri[s]], up = L.up[ri[s]];
                double d = dy[s];
                if (up > OSQP_INFTY * MIN_SCALING) d = (lo < -OSQP_INFTY * MIN_SCALING) ? 0.0 : cmin(d, 0.0);
                else if (lo < -OSQP_INFTY * MIN_SCALING) d = cmax(d, 0.0);
                if (ok) {
                    mx[0] = cmax(mx[0], fabs(ei * pr));
                    mx[2] = cmax(mx[2], fabs(ei * zi));
                    mx[3] = cmax(mx[3], fabs(ei * ax));
                    mx[7] = cmax(mx[7], fabs(pr));
                    mx[9] = cmax(mx[9], fabs(zi));
                    mx[10] = cmax(mx[10], fabs(ax));
                    mx[14] = cmax(mx[14], fabs(unscale ? Ev[s] * d : d));
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
            // q' dx with the out-of-line phases' column-per-thread order (padded column tid)
            if (tid < npad && p.pad_var[tid] >= 0) sm[1] = L.qv[tid] * L.dx[tid];
            block_max<TD, 17>(mx, L.red);
            block_sum<TD, 2>(sm, L.red);
            Res R_;
            if (unscale) {
                R_.pri = mx[0]; R_.dua = cinv * mx[1];
                R_.nz = mx[2]; R_.nax = mx[3]; R_.nq = mx[4]; R_.naty = mx[5]; R_.npx = mx[6];
            } else {
                R_.pri = mx[7]; R_.dua = mx[8];
                R_.nz = mx[9]; R_.nax = mx[10]; R_.nq = mx[11]; R_.naty = mx[12]; R_.npx = mx[13];
            }
            R_.rpri = mx[7]; R_.rdua = mx[8]; R_.rz = mx[9]; R_.rax = mx[10]; R_.rq = mx[11]; R_.raty = mx[12];
            R_.rpx = mx[13];
            if (m == 0) R_.pri = 0.0;
            if (tid == 0) R_.save(L.res);
            if (can_check) {
                int st = MPCQP_UNSOLVED_;
                double obj = 0.0;
                bool done = false;
                if (R_.pri > OSQP_INFTY || R_.dua > OSQP_INFTY) {
                    st = MPCQP_NON_CVX_;
                    obj = __builtin_nan("");
                    done = true;
                } else {
                    const bool prim_ok = m == 0 || R_.pri < p.eps_abs + p.eps_rel * cmax(R_.nz, R_.nax);
                    double mxd = cmax(cmax(R_.nq, R_.naty), R_.npx);
                    if (unscale) mxd *= cinv;
                    const bool dual_ok = R_.dua < p.eps_abs + p.eps_rel * mxd;
                    bool prim_inf = false, dual_inf = false;
                    if (!prim_ok || !dual_ok) {  // infeasibility certificates (uniform branch)
                        __syncthreads();  // the projected delta y
                        const double norm_dy = mx[14], norm_dx = mx[15], epi = p.eps_pinf, edi = p.eps_dinf;
                        double na[1] = {0.0};
                        double a = 0.0;
#pragma unroll
                        for (int k = 0; k < K; ++k) {
                            const unsigned e = cg.e[k];
                            a += lds_at(e & 0xFFFFu) * lds_at((e >> 16) - wbase + dYbase);
                        }
                        if (cv) na[0] = fabs(unscale ? a * (1.0 / Dv) : a);
                        bool viol = false;
#pragma unroll
                        for (int s = 0; s < RS; ++s) {
                            if (!(tid + s * TD < m)) continue;
                            const double ar = unscale ? adx[s] * (1.0 / Ev[s]) : adx[s];
                            const double lo = L.lo[ri[s]], up = L.up[ri[s]];
                            if ((up < OSQP_INFTY * MIN_SCALING && ar > edi * norm_dx) ||
                                (lo > -OSQP_INFTY * MIN_SCALING && ar < -edi * norm_dx))
                                viol = true;
                        }
                        block_max<TD, 1>(na, L.red);
                        viol = block_any<TD>(viol, L.flag);
                        const double cs = unscale ? cval : 1.0;
                        prim_inf = !prim_ok && m != 0 && norm_dy > epi && sm[0] < epi * norm_dy && na[0] < epi * norm_dy;
                        dual_inf = !dual_ok && norm_dx > edi && sm[1] < cs * edi * norm_dx && mx[16] < cs * edi * norm_dx &&
                                   !viol;
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
            Res R_;
            R_.restore(L.res);
            const double pr = R_.rpri / (cmax(R_.rz, R_.rax) + DIVISION_TOL);
            const double du = R_.rdua / (cmax(cmax(R_.rq, R_.raty), R_.rpx) + DIVISION_TOL);
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
        update_info_nl<TD>(p.self, b, cinv);
        info_iter = iter;
        status = check_termination_nl<TD>(p.self, b, cval, cinv, 0);
    }
    const bool has_sol = !(status == MPCQP_PRIMAL_INFEASIBLE_ || status == MPCQP_PRIMAL_INFEASIBLE_INACCURATE_ ||
                           status == MPCQP_DUAL_INFEASIBLE_ || status == MPCQP_DUAL_INFEASIBLE_INACCURATE_ ||
                           status == MPCQP_NON_CVX_);
    if (has_sol) objective_nl<TD>(p.self, cinv);
    if (status == MPCQP_UNSOLVED_) {
        status = check_termination_nl<TD>(p.self, b, cval, cinv, 1);
        if (status == MPCQP_UNSOLVED_) status = MPCQP_MAX_ITER_REACHED_;
    }
    finalize_nl<TD>(p.self, b, xo, yo, cinv, rho, status, info_iter, rho_updates, p.ostat, p.oiter);
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

// The dense kernel's LDS: the base carve, then bc, v2p and the pivot buffers.
size_t lds_dense_bytes(const KParams& p) {
    return (lds_base_bytes(p) + 15) / 16 * 16 + sizeof(double) * (size_t)dense_extra_doubles(kDenseR);
}

template <int R, int K, int RS, int KPK>
static hipError_t go_d(const KParams& p, long B, double* xo, double* yo, int fo, hipStream_t st, KernelRef* ref) {
    auto k = k_solve_d<R, K, RS, KPK>;
    const size_t lds = lds_dense_bytes(p);
    if (ref) { *ref = {(const void*)k, TD, lds}; return hipSuccess; }
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3((unsigned)B), dim3(TD), lds, st, p, xo, yo, fo);
    return hipGetLastError();
}

hipError_t launch_solve_dense(const KParams& p, long B, double* xo, double* yo, int factor_only, hipStream_t st,
                              KernelRef* ref) {
    switch (p.variant) {
        case 16: return go_d<kDenseR, 6, 1, 4>(p, B, xo, yo, factor_only, st, ref);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace mpcqp
