// solve_heavy.hip -- the latency form of the ADMM solve: ONE 512-thread workgroup per QP, alone on
// its CU, for the instances that set a batch's length (variant 19, k_setup_solve_h / k_solve_h).
//
// A cfg-2 batch (SURVEY.md §8 configs[1], B = 1024) lasts as long as its slowest instance: ~350
// ADMM iterations against a mean of 63.  The four-wave kernel (solve_wave.hip,
// variant 17) is built for throughput -- two instances per CU, the three-phase block solve
// x~ = L^-T D^-1 L^-1 b in four barrier intervals -- and runs that instance at ~2,400 cycles an
// iteration.  This kernel trades throughput for latency on one instance:
//
//   x~ = M b with M = K^-1 held explicitly, in registers: lane (row pair, segment) keeps rows
//   r0, r1 of M over 14 columns of one block (blocks of <= 28 real columns, two segments each;
//   ceil(bsize_k / 2) row pairs per block x 8 segments <= 448 lanes), 28 FMAs per lane and an
//   8-lane DPP sum -- one phase instead of three.  The rhs is written in a segment layout whose
//   eight 14-double runs start 18 doubles apart, so a wave's eight segment reads hit disjoint
//   LDS banks (packed at 16 apart they conflicted 4-way: the product phase cost 1,160 cycles
//   against 780, tools/micro/heavy_micro.hip, profiles/r6/heavy_micro*.txt).
//
// One iteration, three barrier intervals:
//   rhs   (thread pc < npad)  x = a x~ + (1 - a) x_prev (the previous iteration's x~), then
//                             b = sigma x - q + A'(rho z - y)                    -> rbs (LDS)
//   prod  (lane (rp, sg))     x~[r] = sum over the 8 segments of M[r][seg] b[seg]  -> xt  (LDS)
//   rows  (thread i < m)      z~ = A x~, relaxation, projection, y, w = rho z - y  -> w   (LDS)
// M is formed after every factorisation (factorize_w4 with 512 threads: the four-wave kernel's
// factor, bit for bit) as M_ab = sum_{k >= max(a, b)} L_ka' S_k^{-1} L_kb  (L_kk = I, L_kj = G_kj:
// the G blocks, rows < amax), each lane its own 28 entries, from the S_k^{-1} tiles and the G
// copy in LDS.  Termination checks, rho adaptation, infeasibility and the final unscaling are
// the four-wave kernel's (solve_wave.hip::solve_w4_body), over 512 threads.  Results equal the
// oracle's (OSQP 0.6) in status and iteration count; the dense product rounds differently from
// the three-phase form, so x agrees with variant 17 to rounding, not bit for bit.
//
// Reference semantics: OSQP 0.6 osqp_solve, behind Control/MPC/mpc_kinematics.py:194-198.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "setup_r.h"
#include "solve_phases.h"
#include "wave_util.h"

namespace mpcqp {

#ifdef MPCQP_EXPERIMENTAL  // measured and not taken: the experimental builds only
constexpr int TH = 512;    // threads per instance
constexpr int HSEG = 14;   // columns per segment (two per block of <= 28 real columns)
constexpr int HSTR = 18;   // doubles between segments in the rhs layout (bank-spread)
constexpr int HRP = 56;    // row pairs at most (4 blocks x 14)

// the S_k^{-1} tiles after the common carve, then the rhs by segment
__host__ __device__ inline size_t lds_h_sg(const KParams& p) { return 16 * ((lds_base_bytes(p) + 15) / 16); }
// block_max_sum_tr over eight waves needs 4 * 8 * 5 + 8 * 2 + 17 doubles of scratch: more than the
// carve's red[128] (it ran into res and the phase timers), so the check reduces in its own
constexpr int HRED = 200;
size_t lds_heavy_bytes(const KParams& p) {
    return lds_h_sg(p) + sizeof(double) * ((size_t)p.nb * SS + 8 * HSTR + HRED + 8);
}

// the factorisation of the four-wave kernel on 512 threads (solve_phases.h::factorize_w4<, 512>)
__device__ __noinline__ bool factorize_h_nl(const KParams* gp, long b, double rho, double* Sg) {
    KPc& p = kconst(gp);
    SL2 c = carve(p);
    return factorize_w4<false, TH>(p, c.L, rho, p.H + b * (long)p.nb * SS, Sg, p.F + b * (long)p.nb * SS);
}

// The lane's row pair: block a, rows i0, i0 + 1 of it (i0 + 1 may be past bsize[a]: no row).
struct HRow {
    int a, i0, n;  // block, first row, rows (1 or 2; 0: no row pair)
};
__device__ __forceinline__ HRow h_row_pair(const KParams& p, int rp) {
    HRow r{0, 0, 0};
    int base = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int bs = p.bsize[k], np = (bs + 1) >> 1;
        if (rp >= base && rp < base + np) {
            r.a = k;
            r.i0 = 2 * (rp - base);
            r.n = min(2, bs - r.i0);
        }
        base += np;
    }
    return r;
}

// Row i of block a of M over the 14 columns [c0, c0 + 14) of block bq (zeros past bsize[bq]):
//   sum_{k >= max(a, bq)} (L_ka' S_k^{-1} L_kb)[i][c]
// S: the S_k^{-1} tiles (LDS, row-major S x S), gl: the G copy (pair k (k - 1) / 2 + j at
// pair * 8 S, rows < amax nonzero, padded to 8).  QR >= amax.
template <int QR>
__device__ __forceinline__ void h_form_row(const KParams& p, const double* Sg, const double* gl, int a, int i,
                                           int bq, int c0, double (&out)[HSEG]) {
    const int amax = p.amax;
    auto G = [&](int k, int j) __attribute__((always_inline)) { return gl + (k * (k - 1) / 2 + j) * 8 * S; };
#pragma unroll
    for (int c = 0; c < HSEG; ++c) out[c] = 0.0;
#pragma unroll 1
    for (int k = max(a, bq); k < 4; ++k) {
        const double* Tk = Sg + k * SS;
        // the left factor's coefficients over the rows p of S_k^{-1}: unit row i (k == a), or
        // G_ka[p][i], p < amax
        double gi[QR];
#pragma unroll
        for (int q = 0; q < QR; ++q) gi[q] = (k > a && q < amax) ? G(k, a)[q * S + i] : 0.0;
        if (k == bq) {  // L_kb = I: sum_p coef_p S_k^{-1}[p][c0 + c]
            if (k == a) {
#pragma unroll
                for (int c = 0; c < HSEG; c += 2) {
                    double v0, v1;
                    ld2(Tk + i * S + c0 + c, v0, v1);
                    out[c] += v0;
                    out[c + 1] += v1;
                }
            } else {
#pragma unroll
                for (int q = 0; q < QR; ++q) {
                    if (q < amax) {
#pragma unroll
                        for (int c = 0; c < HSEG; c += 2) {
                            double v0, v1;
                            ld2(Tk + q * S + c0 + c, v0, v1);
                            out[c] += gi[q] * v0;
                            out[c + 1] += gi[q] * v1;
                        }
                    }
                }
            }
        } else {  // k > bq: sum_q V[q] G_kb[q][c0 + c], V[q] = sum_p coef_p S_k^{-1}[p][q]
            double V[QR];
#pragma unroll
            for (int q = 0; q < QR; ++q) {
                double v = 0.0;
                if (q < amax) {
                    if (k == a) {
                        v = Tk[i * S + q];
                    } else {
#pragma unroll
                        for (int pp = 0; pp < QR; ++pp)
                            if (pp < amax) v += gi[pp] * Tk[pp * S + q];
                    }
                }
                V[q] = v;
            }
            const double* Gb = G(k, bq);
#pragma unroll
            for (int q = 0; q < QR; ++q) {
                if (q < amax) {
#pragma unroll
                    for (int c = 0; c < HSEG; c += 2) {
                        double v0, v1;
                        ld2(Gb + q * S + c0 + c, v0, v1);
                        out[c] += V[q] * v0;
                        out[c + 1] += V[q] * v1;
                    }
                }
            }
        }
    }
    const int bsq = p.bsize[bq];
#pragma unroll
    for (int c = 0; c < HSEG; ++c)
        if (c0 + c >= bsq) out[c] = 0.0;
}

// K: row-list length, KC: column-list length, KPK: P terms per column, QR >= amax.
template <int K, int KC, int KPK, int QR>
__device__ __forceinline__ void solve_h_body(const KParams& p, double* __restrict__ xo, double* __restrict__ yo) {
    const int tid = threadIdx.x;
    const long b = instance_of(p);
    const int n = p.n, m = p.m, npad = p.npad, nnzP = p.nnzP, nnzA = p.nnzA;
    SL2 C = carve(p);
    SLds& L = C.L;
    extern __shared__ __attribute__((aligned(16))) double smh[];
    double* const Sg = smh + lds_h_sg(p) / sizeof(double);  // S_k^{-1} tiles
    double* const rbs = Sg + p.nb * SS;                       // rhs by segment (HSTR apart)
    double* const hred = rbs + 8 * HSTR;                      // the check's reduction scratch (HRED)
    const double* Hg = p.H + b * (long)p.nb * SS;

    if (p.err[b]) {
        for (int j = tid; j < n; j += TH) if (xo) xo[b * n + j] = __builtin_nan("");
        for (int i = tid; i < m; i += TH) if (yo) yo[b * m + i] = __builtin_nan("");
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
    auto cscal = [&](int k) __attribute__((always_inline)) { return opaque_gptr(p.scal + b * 4)[k]; };
    double rho = p.scal[b * 4 + 2];
    const double sigma = p.sigma, alpha = p.alpha;
    const bool warm = p.warm_start != 0;
    for (int e = tid; e < nnzA; e += TH) L.Acsc[e] = p.Ax[b * nnzA + e];
    if (tid == 0) L.Acsc[nnzA] = 0.0;
    for (int v = tid; v < nnzP; v += TH) L.Pv[v] = p.Px[b * nnzP + v];
    if (tid == 0) L.Pv[nnzP] = 0.0;
    const int mp = solve_mpad(m);
    for (int i = tid; i < mp; i += TH) {
        const bool in = i < m;
        L.lo[i] = in ? p.l[b * m + i] : 0.0;
        L.up[i] = in ? p.u[b * m + i] : 0.0;
        L.ct[i] = in ? p.ct[b * m + i] : 0;
        C.Z[i] = (in && warm) ? p.z[b * m + i] : 0.0;
    }
    for (int pc = tid; pc < npad; pc += TH) {
        L.qv[pc] = p.q[b * npad + pc];
        C.X[pc] = warm ? p.x[b * npad + pc] : 0.0;
    }
    for (int e = tid; e < 8 * HSTR; e += TH) rbs[e] = 0.0;
    if (tid < 16) L.res[tid] = 0.0;
    if (tid < 4) L.flag[tid] = 0;

    int status = MPCQP_UNSOLVED_, rho_updates = 0, iter = 0, info_iter = 0;
    bool can_check = false, need_factor = true;
    const unsigned abase = lds_addr(L.Acsc), wbase = lds_addr(L.w), xbase = lds_addr(L.xt);
    const unsigned Xbase = lds_addr(C.X);
    // the lane's dense rows of M (product phase): row pair rp = tid / 8, segment sg = tid % 8
    const int rp = tid >> 3, sg = tid & 7, bq = sg >> 1, c0 = HSEG * (sg & 1);
    const HRow hr = h_row_pair(p, rp);
    const bool prow = rp < HRP && hr.n > 0;
    const int r0 = hr.a * S + hr.i0, r1 = hr.a * S + hr.i0 + 1;
    double Mr[2][HSEG];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int c = 0; c < HSEG; ++c) Mr[r][c] = 0.0;
    GatherW<K> rg;
    GatherW<KC> cg;
    PH(5)
    for (;;) {
        // (the lane's identity through an empty asm: solve_w4_body's OPQ -- the addresses formed
        // at run starts, refactorisations and checks are not held across the solve loop)
        const int tid = opaque_v(threadIdx.x);
        const int pc = tid;                // the lane's column (rhs, checks): pc < npad
        const int ri = min(tid, mp - 1);   // the lane's row: lanes past the padded rows repeat the last
        const bool colw = pc < npad;
        __syncthreads();
        if (need_factor) {
            need_factor = false;
            if (iter > 0) {
                const auto yp = opaque_gptr(p.y + b * m);
                for (int i = tid; i < m; i += TH) yp[i] = L.ys[i];
                __syncthreads();  // every ys read is done before the factorisation's scratch overwrites it
            }
            const bool ok = factorize_h_nl(p.self, b, rho, Sg);
            if (tid == 0) p.ffresh[b] = 0;  // (the workspace Si tiles are not this factor's)
            if (!ok) {
                if (iter == 0) {
                    if (xo) for (int j = tid; j < n; j += TH) opaque_ptr(xo + b * n)[j] = __builtin_nan("");
                    if (yo) for (int i = tid; i < m; i += TH) opaque_ptr(yo + b * m)[i] = __builtin_nan("");
                    if (tid == 0) fail_status(p, b);
                    return;
                }
                status = MPCQP_NON_CVX_;
                can_check = true;
                break;
            }
            __syncthreads();
            const bool have_y = iter > 0 || warm;
            {
                const auto yp = opaque_gptr(p.y + b * m);
                for (int i = tid; i < mp; i += TH) L.ys[i] = (have_y && i < m) ? yp[i] : 0.0;
            }
            constexpr int NP = 6;
            for (int o = tid; o < (NP + 1) * 8 * S; o += TH) {
                const int q = o >> 8, t = (o >> 5) & 7;
                L.gl[o] = (q < NP && t < p.amax) ? Hg[(long)q * p.amax * S + (o & 255)] : 0.0;
            }
            __syncthreads();
            if (prow) {
                h_form_row<QR>(p, Sg, L.gl, hr.a, hr.i0, bq, c0, Mr[0]);
                if (hr.n > 1) {
                    h_form_row<QR>(p, Sg, L.gl, hr.a, hr.i0 + 1, bq, c0, Mr[1]);
                } else {
#pragma unroll
                    for (int c = 0; c < HSEG; ++c) Mr[1][c] = 0.0;
                }
            }
            PH(0)
        }
        // ---- run state ----
        if (colw) cg.load(p.gcol + pc, npad, abase, wbase);
        else cg.clear(abase + 8u * nnzA, wbase);
        if (ri < m) rg.load(p.grow + ri, m, abase, xbase);
        else rg.clear(abase + 8u * nnzA, xbase);
        const bool colv = colw && p.pad_var[pc] >= 0;
        double X = colw ? C.X[pc] : 0.0, DX = 0.0;
        const double Q = colw ? L.qv[pc] : 0.0;
        double ca[KC];
#pragma unroll
        for (int k = 0; k < KC; ++k) ca[k] = lds_at(cg.e[k] & 0xFFFFu);
        // the rhs slot of the column in the segment layout (columns past 28 of a block: none)
        const int cb = pc & (S - 1), chalf = cb >= HSEG;
        const int bslot = (colw && cb < 2 * HSEG) ? HSTR * (2 * (pc >> 5) + chalf) + cb - HSEG * chalf : -1;
        const double r_hi = RHO_EQ_OVER_RHO_INEQ * rho;
        double y = L.ys[ri], Z = C.Z[ri], dy = 0.0;
        double av[K];
#pragma unroll
        for (int k = 0; k < K; ++k) av[k] = lds_at(rg.e[k] & 0xFFFFu);
        const double rlo = L.lo[ri], rup = L.up[ri];
        const signed char cl = L.ct[ri];
        const double rv = cl < 0 ? RHO_MIN : (cl > 0 ? r_hi : rho);
        const double rvi = cl < 0 ? 1.0 / RHO_MIN : (cl > 0 ? 1.0 / r_hi : 1.0 / rho);
        const bool rows_wave = tid < mp;
        if (rows_wave) L.w[ri] = rv * Z - y;
        int stop_at = p.max_iter;
        if (p.check_term) stop_at = min(stop_at, (iter / p.check_term + 1) * p.check_term);
        if (p.adaptive_rho && p.rho_interval) stop_at = min(stop_at, (iter / p.rho_interval + 1) * p.rho_interval);
        bool pend = false;  // xt holds an x~ whose x update the rhs has not applied yet
        // the loop's scalar constants in VGPRs (through an empty asm): held in SGPRs, the
        // compiler spilled them to VGPR lanes and read all sixteen back (v_readlane) at every
        // use in the loop -- 32 reloads an iteration
        double al = alpha, oma = 1.0 - alpha, sg_ = sigma;
        asm volatile("" : "+v"(al), "+v"(oma), "+v"(sg_));
        __syncthreads();
        PH(5)
        while (iter < stop_at) {
            ++iter;
            // rhs: x = a x~ + (1 - a) x_prev (the previous iteration's), b = sigma x - q + A' w
            if (colw) {
                double wv[KC];
#pragma unroll
                for (int k = 0; k < KC; ++k) wv[k] = lds_at(cg.e[k] >> 16);
                const double xtv = L.xt[pc];
                if (pend && colv) X = al * xtv + oma * X;  // (padding: x stays 0)
                double v = sg_ * X - Q;
#pragma unroll
                for (int k = 0; k < KC; ++k) v += ca[k] * wv[k];
                if (bslot >= 0) rbs[bslot] = colv ? v : 0.0;
            }
            pend = true;
            __syncthreads();
            PH(1)
            // x~ = M b: the lane's two rows over its segment, 8-lane sums (segments 0 / 1 store)
            if (prow) {
                double bv[HSEG];
#pragma unroll
                for (int c = 0; c < HSEG; c += 2) ld2(rbs + HSTR * sg + c, bv[c], bv[c + 1]);
                double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
#pragma unroll
                for (int c = 0; c < HSEG; c += 2) {
                    a0 += Mr[0][c] * bv[c];
                    a1 += Mr[0][c + 1] * bv[c + 1];
                    a2 += Mr[1][c] * bv[c];
                    a3 += Mr[1][c + 1] * bv[c + 1];
                }
                const double s0 = reduce8(a0 + a1), s1 = reduce8(a2 + a3);
                if (sg == 0) L.xt[r0] = s0;
                if (sg == 1 && hr.n > 1) L.xt[r1] = s1;
            }
            __syncthreads();
            PH(2)
            // rows: z~ = A x~ ; relaxed + projected z ; y ; next w
            if (rows_wave) {
                double xv[K];
#pragma unroll
                for (int k = 0; k < K; ++k) xv[k] = lds_at(rg.e[k] >> 16);
                double zt = av[0] * xv[0];
#pragma unroll
                for (int k = 1; k < K; ++k) zt += av[k] * xv[k];
                const double zr = al * zt + oma * Z;
                const double zn = __builtin_fmin(__builtin_fmax(zr + rvi * y, rlo), rup);
                const double dd = rv * (zr - zn);
                Z = zn;
                dy = dd;
                y += dd;
                L.w[ri] = rv * zn - y;
            }
            __syncthreads();
            PH(3)
        }
        // the last iteration's x update, then the run state back to LDS (dx aliases xt: mode 2)
        if (colw) {
            const double xo_ = X;
            if (pend && colv) X = al * L.xt[pc] + oma * X;
            DX = X - xo_;
        }
        __syncthreads();  // every x~ read before dx overwrites it
        if (colw) { lds_put(C.X, pc, X); lds_put(L.dx, pc, DX); }
        if (rows_wave) { lds_put(L.ys, ri, y); lds_put(C.Z, ri, Z); lds_put(C.dY, ri, dy); }
        __syncthreads();
        can_check = p.check_term && (iter % p.check_term == 0);
        const bool do_rho = p.adaptive_rho && p.rho_interval && (iter % p.rho_interval == 0);
        if (!can_check && !do_rho) break;
        info_iter = iter;
        bool stop = false;
        {
            // the check (solve_w4_body's, one column per thread pc < npad, one row per thread)
            const int col = colw ? pc : -1;
            const bool cv = colv;
            GatherW<KC> cgk;
            GatherW<KPK> pg;
            if (col >= 0) {
                cgk.load(p.gcol + col, npad, abase, wbase);
                pg.load(p.gpsym + col, npad, lds_addr(L.Pv), Xbase);
            } else {
                cgk.clear(abase + 8u * nnzA, wbase);
                pg.clear(lds_addr(L.Pv) + 8u * nnzP, Xbase);
            }
            const int oz = opaque_zero();
            const double Dv = col >= 0 ? opaque_gptr(p.D + b * npad)[col] : 1.0;
            const double Ev = ri < m ? opaque_gptr(p.E + b * m)[ri] : 1.0;
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
            {  // the thread's column: P x, A' y, P dx, and the delta x norm
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
                    const unsigned e = cgk.e[k];
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
                block_max_sum_tr<TH, 17, 2>(mx, sm, hred);
            } else {
                double m10[10] = {mx[0], mx[1], mx[2], mx[3], mx[4], mx[5], mx[6], mx[14], mx[15], mx[16]};
                block_max_sum_tr<TH, 10, 2>(m10, sm, hred);
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
                                const unsigned e = cgk.e[k];
                                a += lds_at(e & 0xFFFFu) * lds_at((e >> 16) - wbase + dYbase);
                            }
                            if (cv) na[0] = fabs(unscale ? a * (1.0 / Dv) : a);
                            block_max<TH, 1>(na, L.red);
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
                            dual_inf = !block_any<TH>(viol, L.flag);
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
        update_info_nl<TH>(p.self, b, cinv);
        info_iter = iter;
        status = check_termination_nl<TH>(p.self, b, cval, cinv, 0);
    }
    const bool has_sol = !(status == MPCQP_PRIMAL_INFEASIBLE_ || status == MPCQP_PRIMAL_INFEASIBLE_INACCURATE_ ||
                           status == MPCQP_DUAL_INFEASIBLE_ || status == MPCQP_DUAL_INFEASIBLE_INACCURATE_ ||
                           status == MPCQP_NON_CVX_);
    if (has_sol) objective_nl<TH>(p.self, cinv);
    if (status == MPCQP_UNSOLVED_) {
        status = check_termination_nl<TH>(p.self, b, cval, cinv, 1);
        if (status == MPCQP_UNSOLVED_) status = MPCQP_MAX_ITER_REACHED_;
    }
    finalize_nl<TH>(p.self, b, xo, yo, cinv, rho, status, info_iter, rho_updates, p.ostat, p.oiter);
#ifdef MPCQP_PHASE_PROF
    if (prof) {
        __syncthreads();
        PH(5)
        if (tid == 0) {
#pragma unroll
            for (int k = 0; k < 6; ++k) p.prof[b * kProfSlots + k] = L.pacc[k];
#pragma unroll
            for (int k = 8; k < 15; ++k) p.prof[b * kProfSlots + k] = L.pacc[k];
            p.prof[b * kProfSlots + 6] = clock64() - t0c;
            p.prof[b * kProfSlots + 7] = wall_clock64() - t0w;
            p.prof[b * kProfSlots + 15] = t0w;
        }
    }
#endif
#undef PH
}

template <int K, int KC, int KPK, int QR>
__global__ __launch_bounds__(TH, 1) void k_solve_h(KParams p, double* __restrict__ xo, double* __restrict__ yo,
                                                   int /*factor_only: the four-wave kernel's FO launch*/) {
    solve_h_body<K, KC, KPK, QR>(p, xo, yo);
    extern __shared__ __attribute__((aligned(16))) double sm[];
    order_epilogue<TH>(p, (int*)sm);
}

// setup (setup_r.h with 512 threads: one column and one row per thread) + solve
template <int K, int KC, int KPK, int QR, int SK>
__global__ __launch_bounds__(TH, 1) void k_setup_solve_h(KParams p, const double* __restrict__ Px_in,
                                                         const double* __restrict__ Ax_in,
                                                         const double* __restrict__ q_in,
                                                         const double* __restrict__ l_in,
                                                         const double* __restrict__ u_in, double* __restrict__ xo,
                                                         double* __restrict__ yo) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    setup_r_body<TH, SK, 4, 1, 1, 1>(p, instance_of(p), Px_in, Ax_in, q_in, l_in, u_in, sm);
    __syncthreads();
    solve_h_body<K, KC, KPK, QR>(p, xo, yo);
    order_epilogue<TH>(p, (int*)sm);
}

// variant 19's preconditions (solve.hip::variant_fits): the four-wave kernel's plan shape (four
// blocks, no eliminated columns), blocks of at most 28 real columns, one row and one column per
// thread, the fused setup's one A and one P value per thread, the LDS
bool heavy_fits(const KParams& p) {
    KParams q2 = p;
    q2.mode = 2;
    return p.nb == 4 && p.ne == 0 && p.amax <= 8 && p.gkr <= 6 && p.gkc <= 6 && p.pk <= 4 && p.m <= TH &&
           p.npad <= 128 && p.nnzA <= TH && p.nnzP <= TH && p.bsz01 <= 2 * HSEG && p.bsz23 <= 2 * HSEG &&
           lds_heavy_bytes(q2) <= 160 * 1024 && lds_base_bytes(q2) < 65536;
}

// (at least 81 KiB: one workgroup per CU whatever its register count, the instance alone)
size_t heavy_lds(const KParams& p) {
    return std::max({lds_heavy_bytes(p), lds_setup_r_bytes(p.nnzP, p.nnzA, p.npad, p.m, TH), (size_t)81 * 1024});
}

hipError_t launch_solve_heavy(const KParams& p, long B, double* xo, double* yo, int factor_only, hipStream_t st,
                              KernelRef* ref) {
    auto k = p.amax <= 5 ? k_solve_h<6, 6, 4, 5> : k_solve_h<6, 6, 4, 8>;
    const size_t lds = heavy_lds(p);
    if (ref) { *ref = {(const void*)k, TH, lds}; return hipSuccess; }
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3((unsigned)B), dim3(TH), lds, st, p, xo, yo, factor_only);
    return hipGetLastError();
}

hipError_t launch_setup_solve_heavy(const KParams& p, long B, const double* Px, const double* Ax, const double* q,
                                    const double* l, const double* u, double* xo, double* yo, hipStream_t st) {
    auto k = p.amax <= 5 ? k_setup_solve_h<6, 6, 4, 5, 6> : k_setup_solve_h<6, 6, 4, 8, 6>;
    const size_t lds = heavy_lds(p);
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3((unsigned)B), dim3(TH), lds, st, p, Px, Ax, q, l, u, xo, yo);
    return hipGetLastError();
}

#endif  // MPCQP_EXPERIMENTAL

}  // namespace mpcqp
