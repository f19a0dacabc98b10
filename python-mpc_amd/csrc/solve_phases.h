// solve_phases.h -- the parts of the ADMM solve shared by its two kernel shapes
// (solve.hip: one 256-thread workgroup per QP; solve_wave.hip: one 64-lane wave per
// QP): the LDS carve, the in-kernel factorisation of K, the packed gather lists
// and the out-of-line phases (update_info, check_termination with the
// infeasibility certificates, objective, store_solution).  Everything is templated
// on TT, the number of threads working on one QP.
//
// Reference semantics: OSQP 0.6 as called at vehicle_lateral_mpc_slack_increment.py:248
// and Control/MPC/mpc_dynamics.py:396; oracle/osqp_oracle.c restates the same
// algorithm on the CPU.
#pragma once
#include <hip/hip_runtime.h>

#include "device_common.h"

namespace mpcqp {

struct SLds {
    double *Acsc, *Pv, *lo, *up, *qv;
    double *w, *rb, *xt, *ys;        // per-iteration vectors (aliased by the factor scratch)
    double* dx;                      // delta x of the last iteration (rb, or xt in mode 2)
    double* cor;                     // three-phase solve corrections (nb * S, rows < A used)
    double* tv;                      // three-phase solve: D^{-1} L^{-1} b of the wave kernel (npad)
    double* gl;                      // wave kernel: LDS copy of the G blocks (after the vectors in V)
    double *SP, *EK, *DK;            // factorisation scratch (3 tiles)
    double* red;
    double* res;                     // last update_info results (14 doubles)
    long long* pacc;                 // phase timers (diagnostic)
    signed char* ct;
    int* flag;
};

__device__ __forceinline__ double rho_of(signed char t, double rho) {
    return t < 0 ? RHO_MIN : (t > 0 ? RHO_EQ_OVER_RHO_INEQ * rho : rho);
}

// v[j] for a uniform j in [0, 16) without demoting v to scratch (a register array
// indexed by a runtime value would be): a scalar switch
__device__ __forceinline__ double pick16(const double (&v)[16], int j) {
    switch (j) {
#define C(k) case k: return v[k];
        C(0) C(1) C(2) C(3) C(4) C(5) C(6) C(7) C(8) C(9) C(10) C(11) C(12) C(13) C(14)
#undef C
        default: return v[15];
    }
}
__device__ __forceinline__ void put16(double (&v)[16], int j, double x) {
    switch (j) {
#define C(k) case k: v[k] = x; break;
        C(0) C(1) C(2) C(3) C(4) C(5) C(6) C(7) C(8) C(9) C(10) C(11) C(12) C(13) C(14)
#undef C
        default: v[15] = x;
    }
}

// Row i's columns [0, 16) at src (a row of a row-major S x S tile, from column 16 h) into
// v, read as 8 ds_read_b128 in the order column pair s ^ (i & 7) and put back in column
// order by a three-stage conditional-swap network.  In column order every lane of a 16-lane
// group of one read hits the same four banks (the rows are 256 bytes apart: 16-way, 512
// LDS cycles per wave for the 8 reads); rotated, the group's rows spread over the eight
// pairs' bank quads (2-way, 64 cycles; tools/lds_banks.py --swizzle).  The tile layout
// is unchanged.  st_row16 is the same for the store-back.
// The network's swaps are explicit v_cndmask_b32 on the lane mask (the compiler, given
// selects between the values, turned them into a scratch array indexed by m)
__device__ __forceinline__ unsigned sel32(const unsigned long long mk, const unsigned a, const unsigned b) {
    unsigned r;
    asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(mk));
    return r;  // mk's lane bit ? b : a
}
__device__ __forceinline__ double seld(const unsigned long long mk, const double a, const double b) {
    const unsigned lo = sel32(mk, (unsigned)__double2loint(a), (unsigned)__double2loint(b));
    const unsigned hi = sel32(mk, (unsigned)__double2hiint(a), (unsigned)__double2hiint(b));
    return __hiloint2double((int)hi, (int)lo);
}
#define MPCQP_CSW(mk, a, b)                \
    {                                      \
        const double2 t_ = a;              \
        a.x = seld(mk, a.x, b.x);          \
        a.y = seld(mk, a.y, b.y);          \
        b.x = seld(mk, b.x, t_.x);         \
        b.y = seld(mk, b.y, t_.y);         \
    }
#define MPCQP_XOR_PERM8(m, q0, q1, q2, q3, q4, q5, q6, q7)                                           \
    {                                                                                              \
        const unsigned long long s1_ = __builtin_amdgcn_ballot_w64(((m) & 1) != 0);                \
        const unsigned long long s2_ = __builtin_amdgcn_ballot_w64(((m) & 2) != 0);                \
        const unsigned long long s4_ = __builtin_amdgcn_ballot_w64(((m) & 4) != 0);                \
        MPCQP_CSW(s1_, q0, q1) MPCQP_CSW(s1_, q2, q3) MPCQP_CSW(s1_, q4, q5) MPCQP_CSW(s1_, q6, q7) \
        MPCQP_CSW(s2_, q0, q2) MPCQP_CSW(s2_, q1, q3) MPCQP_CSW(s2_, q4, q6) MPCQP_CSW(s2_, q5, q7) \
        MPCQP_CSW(s4_, q0, q4) MPCQP_CSW(s4_, q1, q5) MPCQP_CSW(s4_, q2, q6) MPCQP_CSW(s4_, q3, q7) \
    }
__device__ __forceinline__ void ld_row16(const double* __restrict__ src, const int i, double (&v)[16]) {
    const int m = i & 7;
    double2 q0 = *(const double2*)(src + 2 * (0 ^ m)), q1 = *(const double2*)(src + 2 * (1 ^ m));
    double2 q2 = *(const double2*)(src + 2 * (2 ^ m)), q3 = *(const double2*)(src + 2 * (3 ^ m));
    double2 q4 = *(const double2*)(src + 2 * (4 ^ m)), q5 = *(const double2*)(src + 2 * (5 ^ m));
    double2 q6 = *(const double2*)(src + 2 * (6 ^ m)), q7 = *(const double2*)(src + 2 * (7 ^ m));
    MPCQP_XOR_PERM8(m, q0, q1, q2, q3, q4, q5, q6, q7)  // q_s held pair s ^ m; now pair s
    v[0] = q0.x, v[1] = q0.y, v[2] = q1.x, v[3] = q1.y, v[4] = q2.x, v[5] = q2.y, v[6] = q3.x, v[7] = q3.y;
    v[8] = q4.x, v[9] = q4.y, v[10] = q5.x, v[11] = q5.y, v[12] = q6.x, v[13] = q6.y, v[14] = q7.x, v[15] = q7.y;
}
// sc * v to dst
__device__ __forceinline__ void st_row16(double* __restrict__ dst, const int i, const double sc, const double (&v)[16]) {
    const int m = i & 7;
    double2 q0 = make_double2(sc * v[0], sc * v[1]), q1 = make_double2(sc * v[2], sc * v[3]);
    double2 q2 = make_double2(sc * v[4], sc * v[5]), q3 = make_double2(sc * v[6], sc * v[7]);
    double2 q4 = make_double2(sc * v[8], sc * v[9]), q5 = make_double2(sc * v[10], sc * v[11]);
    double2 q6 = make_double2(sc * v[12], sc * v[13]), q7 = make_double2(sc * v[14], sc * v[15]);
    MPCQP_XOR_PERM8(m, q0, q1, q2, q3, q4, q5, q6, q7)  // q_s = pair s ^ m
#define MPCQP_ST(s) *(double2*)(dst + 2 * ((s) ^ m)) = q##s;
    MPCQP_ST(0) MPCQP_ST(1) MPCQP_ST(2) MPCQP_ST(3) MPCQP_ST(4) MPCQP_ST(5) MPCQP_ST(6) MPCQP_ST(7)
#undef MPCQP_ST
}
#undef MPCQP_XOR_PERM8
#undef MPCQP_CSW

// Gauss-Jordan inverse of the SPD tile T (32 x 32 in LDS) by ONE wave, in place, with a
// copy to Sgk.  Lane (i, h) = (lane % 32, lane / 32) keeps row i, columns [16 h, 16 h + 16)
// in registers.  The in-place Gauss-Jordan matrix of a symmetric input stays symmetric up
// to sign -- M_ij = -M_ji exactly when one of i, j is already pivoted -- so row p is
// published by the lanes that hold column p (one ds_write_b64 per lane and pivot) and the
// 32 pivots need no workgroup barrier.  buf: 2 S doubles.  False on a non-positive pivot.
// npiv: the tile's real rows (plan bsize); the rest are padding at the end -- identity
// rows and columns that pivoting leaves as they are -- so the rolled loop skips their
// pivots (cfg 3's 256-thread kernel: solve 40.1 -> 39.3 ms at B = 16384).
//
// Compact = false: the pivot loop is unrolled (static register indices, fastest; the
// wave kernels can afford its ~200 VGPRs).  Compact = true: a rolled loop whose pivot
// slot is picked with scalar switches (~90 VGPRs), for the 256-thread kernels, where
// the unrolled form costs occupancy in every other phase.
template <bool Compact>
__device__ __forceinline__ bool gj_wave(double* __restrict__ T, double* __restrict__ buf, double* __restrict__ Sgk,
                                        const int npiv = S) {
    const int lane = threadIdx.x & 63, i = lane & 31, h = lane >> 5;
    double v[16];
#pragma unroll
    for (int jj = 0; jj < 16; jj += 2) {
        const double2 t2 = *(const double2*)(T + i * S + 16 * h + jj);
        v[jj] = t2.x;
        v[jj + 1] = t2.y;
    }
    double minpiv = 1.0;  // -1 once a pivot is not positive (NaN-safe running flag)
    // Row scaling deferred: the lane keeps its row as sc * v.  Pivoting row p only sets
    // its scale to 1 / piv (no pass over its elements), so every pivot step is one
    // masked FMA pass; the true values are published per pivot (one multiply) and
    // restored once at the end.  iv = 1 / sc, exactly piv for pivoted rows.
    double sc = 1.0, iv = 1.0;
    // Branch-free pivot step (the rolled loop): after the publish, the pivot, the lane's
    // column entry and the lane's half of row p are read together, so the row's LDS
    // latency overlaps the reciprocal's Newton chain; the pivot row's own lane runs the
    // FMA pass with a zero multiplier (v + (-0) * row == v exactly for finite rows).
    // cfg 3 (256-thread kernel) Gauss-Jordan 868 k -> 767 k cycles per slowest solve (the
    // solve time is the same with the divergent step here: measured A/B, round 2).
    auto pivot = [&](const int p, const int pj) __attribute__((always_inline)) {
        const int ph = p >> 4;
        double* rb = buf + (pj & 1) * S;
        if (h == ph) {
            const double vp = sc * (Compact ? pick16(v, pj) : v[pj]);
            rb[i] = i < p ? -vp : vp;  // row p = +-column p
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const double piv = rb[p];
        const double mi = rb[i];
        double rowv[16];
#pragma unroll
        for (int jj = 0; jj < 16; jj += 2) {
            const double2 r2 = *(const double2*)(rb + 16 * h + jj);
            rowv[jj] = r2.x;
            rowv[jj + 1] = r2.y;
        }
        const double colv = i < p ? -mi : mi;  // M_ip
        minpiv = piv > 0.0 ? minpiv : -1.0;
        // 1 / piv: hardware reciprocal and two Newton steps (full double precision)
        double d = __builtin_amdgcn_rcp(piv);
        d = __builtin_fma(d, __builtin_fma(-piv, d, 1.0), d);
        d = __builtin_fma(d, __builtin_fma(-piv, d, 1.0), d);
        // every other row loses M_ip / piv times row_p (in its own scale); row p keeps
        // its elements and takes the scale 1 / piv
        const bool self = i == p;
        const double cd = self ? 0.0 : (colv * d) * iv;
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) v[jj] = __builtin_fma(-cd, rowv[jj], v[jj]);
        sc = self ? d : sc;
        iv = self ? piv : iv;
        if (h == ph) {
            if (Compact) put16(v, pj, self ? 1.0 : -cd);
            else v[pj] = self ? 1.0 : -cd;
        }
    };
    if constexpr (Compact) {
#pragma unroll 1
        for (int p = 0; p < npiv; ++p) pivot(p, __builtin_amdgcn_readfirstlane(p & 15));
    } else {
        // the unrolled loop keeps the divergent update: measured faster here than the
        // branch-free step (cfg 2 Gauss-Jordan 233 k vs 275 k cycles per solve of the
        // slowest instance), and as fast as a one-pivot lookahead variant (238 k)
        auto pivot_br = [&](const int p, const int pj) __attribute__((always_inline)) {
            const int ph = p >> 4;
            double* rb = buf + (pj & 1) * S;
            if (h == ph) {
                const double vp = sc * v[pj];
                rb[i] = i < p ? -vp : vp;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            double rowv[16];
#pragma unroll
            for (int jj = 0; jj < 16; jj += 2) {
                const double2 r2 = *(const double2*)(rb + 16 * h + jj);
                rowv[jj] = r2.x;
                rowv[jj + 1] = r2.y;
            }
            const double piv = rb[p];
            const double mi = rb[i];
            const double colv = i < p ? -mi : mi;
            minpiv = piv > 0.0 ? minpiv : -1.0;
            double d = __builtin_amdgcn_rcp(piv);
            d = __builtin_fma(d, __builtin_fma(-piv, d, 1.0), d);
            d = __builtin_fma(d, __builtin_fma(-piv, d, 1.0), d);
            const double cd = (colv * d) * iv;
            if (i != p) {
#pragma unroll
                for (int jj = 0; jj < 16; ++jj) v[jj] = __builtin_fma(-cd, rowv[jj], v[jj]);
            } else {
                sc = d;
                iv = piv;
            }
            if (h == ph) v[pj] = i == p ? 1.0 : -cd;
        };
        // the padding pivots (p >= npiv) are skipped by a uniform branch around each unrolled
        // step (an early exit out of the loop broke the unrolled schedule: cfg 2
        // Gauss-Jordan 227 k -> 297 k cycles on the slowest instance).  Skipping one leaves
        // its identity row / column as they are, up to the sign of the zeros the step
        // would have written (-0.0 for +0.0 in padded entries, never read as nonzero).
#pragma unroll
        for (int p = 0; p < S; ++p)
            if (p < npiv) pivot_br(p, p & 15);
    }
#pragma unroll
    for (int jj = 0; jj < 16; jj += 2) {
        const double2 t2 = make_double2(sc * v[jj], sc * v[jj + 1]);
        *(double2*)(T + i * S + 16 * h + jj) = t2;
        *(double2*)(Sgk + i * S + 16 * h + jj) = t2;
    }
    return minpiv > 0.0;
}

// Gauss-Jordan of one tile in two segments, by one wave, in place (the split
// factorisations factorize_w2 / factorize_g).  S_k = D_k - F_k E_k' differs from the
// assembled D_k only in the corner [0, a)^2 of its coupling rows (E_k has a nonzero
// rows), and a pivot step changes an unpivoted entry by terms that do not involve it.
// So SEG 1 pivots rows [a, npiv) of D_k before S_{k-1}^{-1} exists -- its unpivoted
// corner is then the Schur complement of D_k onto the coupling rows -- and SEG 2, once
// F_k is known, adds the correction dl (a x a, row stride 16: -F_k E_k') to that corner
// and pivots rows [0, a); the tile then holds S_k^{-1}.  SEG 1 with a = 0 is the whole
// inverse in gj_wave's natural order.  The steps are gj_wave's (Compact: the rolled,
// branch-free one with scalar-switch register picks, for the 256-thread kernels); the
// pivot order only changes which rows count as pivoted in the sign rule M_ij = -M_ji.
// T (LDS or the workspace) holds true values between the segments (sc = 1 on entry).
// buf: 2 S doubles of LDS.  a <= 16 (a <= 8 for the unrolled SEG 2).
// Rot (unrolled form only): the tile rows are read and written in ld_row16's rotated order.
template <int SEG, bool Compact = false, bool Rot = false>
__device__ __forceinline__ bool gj_seg(double* __restrict__ T, double* __restrict__ buf, const int a, const int npiv,
                                       const double* __restrict__ dl) {
    const int lane = threadIdx.x & 63, i = lane & 31, h = lane >> 5;
    double v[16];
    if constexpr (!Rot || Compact) {
#pragma unroll
        for (int jj = 0; jj < 16; jj += 2) {
            const double2 t2 = *(const double2*)(T + i * S + 16 * h + jj);
            v[jj] = t2.x;
            v[jj + 1] = t2.y;
        }
    } else {
        ld_row16(T + i * S + 16 * h, i, v);
    }
    if (SEG == 2 && h == 0 && i < a) {
#pragma unroll
        for (int jj = 0; jj < 16; ++jj)
            if (jj < a) v[jj] += dl[i * 16 + jj];
    }
    double minpiv = 1.0, sc = 1.0, iv = 1.0;
    auto step = [&](const int p, const int pj, const bool pv) __attribute__((always_inline)) {
        const int ph = p >> 4;
        double* rb = buf + (pj & 1) * S;
        if (h == ph) {
            const double vp = sc * (Compact ? pick16(v, pj) : v[pj]);
            rb[i] = pv ? -vp : vp;  // row p = +-column p
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const double piv = rb[p];
        const double mi = rb[i];
        double rowv[16];
#pragma unroll
        for (int jj = 0; jj < 16; jj += 2) {
            const double2 r2 = *(const double2*)(rb + 16 * h + jj);
            rowv[jj] = r2.x;
            rowv[jj + 1] = r2.y;
        }
        const double colv = pv ? -mi : mi;
        minpiv = piv > 0.0 ? minpiv : -1.0;
        double d = __builtin_amdgcn_rcp(piv);
        d = __builtin_fma(d, __builtin_fma(-piv, d, 1.0), d);
        d = __builtin_fma(d, __builtin_fma(-piv, d, 1.0), d);
        const bool self = i == p;
        if constexpr (Compact) {
            const double cd = self ? 0.0 : (colv * d) * iv;
#pragma unroll
            for (int jj = 0; jj < 16; ++jj) v[jj] = __builtin_fma(-cd, rowv[jj], v[jj]);
            sc = self ? d : sc;
            iv = self ? piv : iv;
            if (h == ph) put16(v, pj, self ? 1.0 : -cd);
        } else {
            const double cd = (colv * d) * iv;
            if (!self) {
#pragma unroll
                for (int jj = 0; jj < 16; ++jj) v[jj] = __builtin_fma(-cd, rowv[jj], v[jj]);
            } else {
                sc = d;
                iv = piv;
            }
            if (h == ph) v[pj] = self ? 1.0 : -cd;
        }
    };
    if constexpr (Compact) {
        if constexpr (SEG == 1) {
#pragma unroll 1
            for (int p = a; p < npiv; ++p) step(p, __builtin_amdgcn_readfirstlane(p & 15), i >= a && i < p);
        } else {
            const bool done = i >= a && i < npiv;
#pragma unroll 1
            for (int p = 0; p < a; ++p) step(p, __builtin_amdgcn_readfirstlane(p & 15), done || i < p);
        }
    } else if constexpr (SEG == 1) {
#pragma unroll
        for (int p = 0; p < S; ++p)
            if (p >= a && p < npiv) step(p, p & 15, i >= a && i < p);
    } else {
        const bool done = i >= a && i < npiv;  // pivoted in SEG 1
#pragma unroll
        for (int p = 0; p < 8; ++p)
            if (p < a) step(p, p, done || i < p);
    }
    if constexpr (!Rot || Compact) {
#pragma unroll
        for (int jj = 0; jj < 16; jj += 2) *(double2*)(T + i * S + 16 * h + jj) = make_double2(sc * v[jj], sc * v[jj + 1]);
    } else {
        st_row16(T + i * S + 16 * h, i, sc, v);
    }
    return minpiv > 0.0;
}

// Assembly of block k's D_k (sigma I + the plan's terms) and E_k (rows < amax) by the
// threads t0, t0 + nt, ...; sync() orders the zeroing before the targets' sums.
// POL: the polish system's row weights (factorize's comment).
template <bool POL, bool DEEP, bool STORE, class KP>
__device__ __forceinline__ void assemble_targets(const KP& p, const SLds& L, const double rho, const int k,
                                                 double* __restrict__ D, double* __restrict__ E, const int t0,
                                                 const int nt);
template <bool POL, bool DEEP, class KP, class Sync>
__device__ __forceinline__ void assemble_block(const KP& p, const SLds& L, const double rho, const int k,
                                               double* __restrict__ D, double* __restrict__ E, const int t0,
                                               const int nt, Sync sync) {
    const int amax = p.amax;
    for (int e = 2 * t0; e < SS; e += 2 * nt) *(double2*)(D + e) = make_double2(0.0, 0.0);
    for (int e = 2 * t0; e < amax * S; e += 2 * nt) *(double2*)(E + e) = make_double2(0.0, 0.0);
    sync();
    if (t0 < S) D[t0 * S + t0] = p.pad_var[k * S + t0] >= 0 ? (POL ? p.delta : p.sigma) : 1.0;
    sync();
    assemble_targets<POL, DEEP, false>(p, L, rho, k, D, E, t0, nt);
}

// The targets' sums (assemble_block).  STORE: the tiles hold zeros and the diagonal
// (sigma, or 1 on padding rows) already, and every target is written once as that
// base value plus its sum (no read: the workspace tiles of factorize_g).
template <bool POL, bool DEEP, bool STORE, class KP>
__device__ __forceinline__ void assemble_targets(const KP& p, const SLds& L, const double rho, const int k,
                                                 double* __restrict__ D, double* __restrict__ E, const int t0,
                                                 const int nt) {
    const int ntgt = p.ntgt;
    const int2* __restrict__ tt = (const int2*)p.tterm;
    // every target has one owner: its terms are summed in plan order.  The wave's first
    // target has the most terms (plan order); the others pad with zero terms to its count.
    const int tb = p.asm_blk_ptr[k], te = p.asm_blk_ptr[k + 1], tmax = p.term_max;
    if (te <= tb) return;
    auto term = [&](const int2 w) __attribute__((always_inline)) {
        const int a = w.x & 0xFFFF, bb = (int)((unsigned)w.x >> 16), r = w.y;
        const double wr = POL ? (double)((L.ct[r] & 1) + ((L.ct[r] >> 1) & 1)) * rho : rho_of(L.ct[r], rho);
        return r < 0 ? L.Pv[a] : wr * L.Acsc[a] * L.Acsc[bb];
    };
    auto add = [&](const int tg, const double acc) __attribute__((always_inline)) {
        if constexpr (STORE) {
            if (tg < SS) D[tg] = ((tg >> 5) == (tg & (S - 1)) ? (POL ? p.delta : p.sigma) : 0.0) + acc;
            else E[tg - SS] = 0.0 + acc;
        } else {
            if (tg < SS) D[tg] += acc;
            else E[tg - SS] += acc;
        }
    };
    int t_rest = tb + t0;
    if constexpr (DEEP) {
        // The count, tile index and first term (the only one for most targets) of the
        // lane's first NI targets, and the further terms of its first target (sorted
        // first: the multi-term ones), are all loaded before any is summed, so the plan's
        // L2 / MALL latency is paid about once per block instead of once per target
        // (two-wave kernel; the extra registers cost the 256-thread kernels' solve loops).
        constexpr int NI = 8, TJ = 6;
        int tn[NI], tg[NI];
        int2 w0[NI], wj[TJ];
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int tc = min(tb + t0 + i * nt, te - 1);
            tn[i] = p.tcnt[__builtin_amdgcn_readfirstlane(tc)];
            tg[i] = p.asm_tgt[tc];
            w0[i] = tt[tc];
        }
        const int tc0 = min(tb + t0, te - 1);
#pragma unroll
        for (int j = 1; j < TJ; ++j) wj[j] = tt[(long)min(j, tmax - 1) * ntgt + tc0];
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int t = tb + t0 + i * nt;
            if (t < te) {
                double acc = 0.0;
                acc += term(w0[i]);
                if (i == 0) {
#pragma unroll
                    for (int j = 1; j < TJ; ++j)
                        if (j < tn[0]) acc += term(wj[j]);
#pragma unroll 1
                    for (int j = TJ; j < tn[0]; ++j) acc += term(tt[(long)j * ntgt + t]);
                } else {
#pragma unroll 1
                    for (int j = 1; j < tn[i]; ++j) acc += term(tt[(long)j * ntgt + t]);
                }
                add(tg[i], acc);
            }
        }
        t_rest = tb + t0 + NI * nt;
    }
    // the (remaining) targets one at a time, the next one's plan loads in flight while
    // the current one is summed
    if (t_rest >= te) return;
    int t = t_rest, tc = min(t, te - 1);
    int tn = p.tcnt[__builtin_amdgcn_readfirstlane(tc)], tg = p.asm_tgt[tc];
    int2 w0 = tt[tc];
#pragma unroll 1
    for (; t < te; t += nt) {
        const int tcn = min(t + nt, te - 1);
        const int tn_n = p.tcnt[__builtin_amdgcn_readfirstlane(tcn)], tg_n = p.asm_tgt[tcn];
        const int2 w0_n = tt[tcn];
        double acc = 0.0;
        acc += term(w0);
#pragma unroll 2
        for (int j = 1; j < tn; ++j) acc += term(tt[(long)j * ntgt + t]);
        add(tg, acc);
        tn = tn_n; tg = tg_n; w0 = w0_n;
    }
}

// The two-wave kernel's factorisation (mode 2, nb = 4, amax <= 8; TT = 128), with the
// Gauss-Jordan pivots that do not wait for the previous block taken off the critical
// path (gj_seg):
//   stage 1, the waves in parallel: wave 0 assembles D_0 and inverts it whole, then
//     assembles D_2 and pivots its rows [amax, 32); wave 1 does the same for D_1, D_3;
//   then for k = 1..3:  F_k = E_k S_{k-1}^{-1} (G_{k,k-1} = -F_k), the corner correction
//     -F_k E_k' and the blocks G_kj = -F_k G_{k-1,j} (j < k-1) from LDS, then wave 0
//     pivots rows [0, amax) of S_k (gj_seg<2>).
// The critical path is 32 + 3 amax pivot steps instead of 4 x 32.  Outputs as mode 2 of
// factorize: S_k^{-1} in Sg (LDS here), G_kj in Hg at pair k(k-1)/2 + j.
template <bool ROT = false, class KP>
__device__ __forceinline__ bool factorize_w2(const KP& p, SLds& L, const double rho, double* __restrict__ Hg,
                                             double* __restrict__ Sg) {
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int amax = p.amax, as = amax * S;
    const long gstride = (long)amax * S;
    // scratch in the aliased vector region: E_0..E_3, F_1..F_3, G_20, the corner, the buffers
    double* const V = L.SP;
    double* const G20 = V + 7 * as;
    double* const dl = V + 8 * as;             // amax x amax, row stride 16
    double* const bufw = dl + 256 + w * 2 * S;  // the wave's Gauss-Jordan publish buffers
    double* const okf = dl + 256 + 4 * S;
    auto Ek = [&](int k) __attribute__((always_inline)) { return V + k * as; };
    auto Fk = [&](int k) __attribute__((always_inline)) { return V + (3 + k) * as; };
    auto wave_sync = []() __attribute__((always_inline)) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
#ifdef MPCQP_PHASE_PROF
    long long tf = clock64();
#define FPH(k) if (tid == 0) { const long long t_ = clock64(); L.pacc[k] += t_ - tf; tf = t_; }
#else
#define FPH(k)
#endif
    bool okw = true;
#pragma unroll 1
    for (int s = 0; s < 2; ++s) {
        const int k = w + 2 * s;
        assemble_block<false, true>(p, L, rho, k, Sg + (long)k * SS, Ek(k), lane, 64, wave_sync);
        wave_sync();
        FPH(8)
        okw = gj_seg<1, false, ROT>(Sg + (long)k * SS, bufw, k ? amax : 0, p.bsize[k], nullptr) && okw;
        FPH(10)
    }
    __syncthreads();
    FPH(11)
#pragma unroll 1
    for (int k = 1; k < 4; ++k) {
        const double* Sp = Sg + (long)(k - 1) * SS;
        const double* E = Ek(k);
        double* F = Fk(k);
        // E_k's nonzero columns are [l0, l0 + bmax) of block k-1 (plan toff / bmax): the
        // products skip its zero columns (same sums, in the same order)
        const int l0 = p.toff[k - 1], bmax = p.bmax;
        for (int o = tid; o < as; o += 128) {
            const int r = o >> 5, j = o & (S - 1);
            double sacc = 0.0;
#pragma unroll 4
            for (int l = l0; l < l0 + bmax; ++l) sacc += E[r * S + l] * Sp[l * S + j];
            F[o] = sacc;
            Hg[(long)(k * (k - 1) / 2 + k - 1) * gstride + o] = -sacc;
        }
        __syncthreads();
        if (tid < amax * amax) {  // S_k = D_k - F_k E_k' on the corner
            const int r = tid / amax, c = tid - r * amax;
            double sacc = 0.0;
#pragma unroll 4
            for (int l = l0; l < l0 + bmax; ++l) sacc += F[r * S + l] * E[c * S + l];
            dl[r * 16 + c] = -sacc;
        }
        // G_kj = -F_k G_{k-1,j}: G_{k-1,k-2} = -F_{k-1}; G_{2,0} kept in LDS for k = 3
#pragma unroll 1
        for (int j = 0; j < k - 1; ++j) {
            const bool adj = j == k - 2;
            const double* Gp = adj ? Fk(k - 1) : G20;
            const double sg = adj ? 1.0 : -1.0;  // G_kj = sg * F_k Gp
            for (int o = tid; o < as; o += 128) {
                const int r = o >> 5, c = o & (S - 1);
                double sacc = 0.0;
#pragma unroll
                for (int l = 0; l < 8; ++l)
                    if (l < amax) sacc += F[r * S + l] * Gp[l * S + c];
                const double g = sg * sacc;
                Hg[(long)(k * (k - 1) / 2 + j) * gstride + o] = g;
                if (k == 2) G20[o] = g;
            }
        }
        __syncthreads();
        FPH(9)
        if (w == 0) okw = gj_seg<2, false, ROT>(Sg + (long)k * SS, bufw, amax, p.bsize[k], dl) && okw;
        __syncthreads();
        FPH(11)
    }
    if (lane == 0) okf[w] = okw ? 1.0 : 0.0;
    __syncthreads();
    FPH(9)
#undef FPH
    return okf[0] > 0.5 && okf[1] > 0.5;
}

// The four-wave kernel's factorisation (solve_wave.hip::k_solve_w4, variant 17: mode 2,
// nb = 4, amax <= 8; TT = 256): factorize_w2 with one wave per block in stage 1 -- wave
// k assembles D_k and pre-pivots it (block 0: the whole inverse), all four at once --
// then the same k = 1..3 chain (F_k, the corner, the G blocks, wave 0's corner pivots).
// The critical path of stage 1 is one block's pivots instead of two.  Same outputs.
// TT = 512 (solve_heavy.hip, the one-instance-per-CU kernel): waves 0-3 run stage 1 and the
// chain exactly as with 256 threads, waves 4-7 join the F / G products (the same sums per
// output element: the factor is bit-identical to the 256-thread one).
template <bool ROT = false, int TT = 256, class KP>
__device__ __forceinline__ bool factorize_w4(const KP& p, SLds& L, const double rho, double* __restrict__ Hg,
                                             double* __restrict__ Sg, double* __restrict__ Fo) {
    static_assert(TT == 256 || TT == 512, "four or eight waves");
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int amax = p.amax, as = amax * S;
    const long gstride = (long)amax * S;
    double* const V = L.SP;
    double* const G20 = V + 7 * as;
    double* const dl = V + 8 * as;              // amax x amax, row stride 16
    double* const bufw = dl + 256 + w * 2 * S;  // the wave's Gauss-Jordan publish buffers
    double* const okf = dl + 256 + 8 * S;
    auto Ek = [&](int k) __attribute__((always_inline)) { return V + k * as; };
    auto Fk = [&](int k) __attribute__((always_inline)) { return V + (3 + k) * as; };
    auto wave_sync = []() __attribute__((always_inline)) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
#ifdef MPCQP_PHASE_PROF
    long long tf = clock64();
#define FPH(k) if (tid == 0) { const long long t_ = clock64(); L.pacc[k] += t_ - tf; tf = t_; }
#else
#define FPH(k)
#endif
    const bool sw = TT == 256 || w < 4;  // a stage-1 wave (wave w: block w)
    // an eliminated column's pivot K_jj is a pivot of the full KKT factorisation too: a
    // non-positive (or NaN) one makes the instance non-convex, as OSQP's LDL' of the
    // quasi-definite matrix would find, even though the reduced blocks may still factor
    bool oke = true;
    if (sw) {
    assemble_block<false, true>(p, L, rho, w, Sg + (long)w * SS, Ek(w), lane, 64, wave_sync);
    wave_sync();
    if (p.ne && lane < S) {
        // eliminated columns (plan.h Plan::eown): the owner lane of block column w S + lane
        // forms K_jj, K_pj of its column j, folds the Schur complement -K_pj^2 / K_jj into its
        // diagonal entry of D_w, and leaves ec = K_pj / K_jj, ed = 1 / K_jj in the instance's F
        // tiles (unused by the three-phase form) for the solve's rhs and x updates
        const int pe = p.eown[w * S + lane];
        if (pe >= 0) {
            const int e = pe - p.nb * S, ne2 = 2 * p.ne;
            const int2* __restrict__ et = (const int2*)p.etterm;
            double kjj = p.sigma, kpj = 0.0;
            for (int j = 0; j < p.eterm_max; ++j) {
                const int2 a = et[(long)j * ne2 + 2 * e], c = et[(long)j * ne2 + 2 * e + 1];
                kjj += a.y < 0 ? L.Pv[a.x] : rho_of(L.ct[a.y], rho) * L.Acsc[a.x & 0xFFFF] * L.Acsc[(unsigned)a.x >> 16];
                kpj += c.y < 0 ? L.Pv[c.x] : rho_of(L.ct[c.y], rho) * L.Acsc[c.x & 0xFFFF] * L.Acsc[(unsigned)c.x >> 16];
            }
            const double ed = 1.0 / kjj, ec = kpj * ed;
            oke = kjj > 0.0 && ed < __builtin_huge_val();
            Sg[(long)w * SS + lane * S + lane] -= kpj * ec;
            Fo[2 * e] = ec;
            Fo[2 * e + 1] = ed;
        }
        wave_sync();
    }
    }
    FPH(8)
    bool okw = true;
    if (sw) {
        okw = gj_seg<1, false, ROT>(Sg + (long)w * SS, bufw, w ? amax : 0, p.bsize[w], nullptr);
        okw = okw && __builtin_amdgcn_ballot_w64(!oke) == 0;
    }
    FPH(10)
    __syncthreads();
    FPH(11)
#pragma unroll 1
    for (int k = 1; k < 4; ++k) {
        const double* Sp = Sg + (long)(k - 1) * SS;
        const double* E = Ek(k);
        double* F = Fk(k);
        const int l0 = p.toff[k - 1], bmax = p.bmax;
        for (int o = tid; o < as; o += TT) {
            const int r = o >> 5, j = o & (S - 1);
            double sacc = 0.0;
#pragma unroll 4
            for (int l = l0; l < l0 + bmax; ++l) sacc += E[r * S + l] * Sp[l * S + j];
            F[o] = sacc;
            Hg[(long)(k * (k - 1) / 2 + k - 1) * gstride + o] = -sacc;
        }
        __syncthreads();
        FPH(9)
        if (w == 0) {
            // wave 0: the corner S_k = D_k - F_k E_k' and its pivots right away (one wave:
            // a wave sync orders the corner before gj_seg reads it)
            if (lane < amax * amax) {
                const int r = lane / amax, c = lane - r * amax;
                double sacc = 0.0;
#pragma unroll 4
                for (int l = l0; l < l0 + bmax; ++l) sacc += F[r * S + l] * E[c * S + l];
                dl[r * 16 + c] = -sacc;
            }
            wave_sync();
            okw = gj_seg<2, false, ROT>(Sg + (long)k * SS, bufw, amax, p.bsize[k], dl) && okw;
        } else {
            // waves 1-3 meanwhile: G_kj = -F_k G_{k-1,j} (j < k-1), off the chain's path
#pragma unroll 1
            for (int j = 0; j < k - 1; ++j) {
                const bool adj = j == k - 2;
                const double* Gp = adj ? Fk(k - 1) : G20;
                const double sg = adj ? 1.0 : -1.0;
                for (int o = tid - 64; o < as; o += TT - 64) {
                    const int r = o >> 5, c = o & (S - 1);
                    double sacc = 0.0;
#pragma unroll
                    for (int l = 0; l < 8; ++l)
                        if (l < amax) sacc += F[r * S + l] * Gp[l * S + c];
                    const double g = sg * sacc;
                    Hg[(long)(k * (k - 1) / 2 + j) * gstride + o] = g;
                    if (k == 2) G20[o] = g;
                }
            }
        }
        __syncthreads();
        FPH(11)
    }
    if (lane == 0) okf[w] = okw ? 1.0 : 0.0;
    __syncthreads();
    FPH(9)
#undef FPH
    return okf[0] > 0.5 && okf[1] > 0.5 && okf[2] > 0.5 && okf[3] > 0.5;
}

// factorize_w4's form for the one-shot kernel on plans whose G blocks have no LDS region of
// their own (one_shot_form 3, the slack layouts): the G blocks go straight into the solve's
// copy gl (pair q at q 8 S, rows < amax; rows amax..7 and pair NP are zero from the kernel's
// start), and F_k, G_20 are read back from there instead of the scratch tiles Fk / G20
// (G_{k,k-1} = -F_k: a sum over negated operands is the negated sum, exactly, so every
// stored value is the workspace form's bit for bit).  Scratch: E_0..E_3 and the wave buffers
// at the start of the carve's V span (w, rb, xt, ys, dY: dead across a factorisation, y parked
// by the caller; one_shot_form checks that they end before gl), the corner correction in red.
template <bool ROT = false, class KP>
__device__ __forceinline__ bool factorize_w4_gl(const KP& p, SLds& L, const double rho, double* __restrict__ Sg,
                                                double* __restrict__ Fo) {
    constexpr int TT = 256;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int amax = p.amax, as = amax * S;
    constexpr long gstride = 8 * S;
    double* const V = L.SP;
    double* const Gl = L.gl;
    double* const dl = L.red;                          // amax x amax, row stride 16
    double* const bufw = V + 4 * as + w * 2 * S;       // the wave's Gauss-Jordan publish buffers
    double* const okf = V + 4 * as + 8 * S;
    auto Ek = [&](int k) __attribute__((always_inline)) { return V + k * as; };
    auto wave_sync = []() __attribute__((always_inline)) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    bool oke = true;
    assemble_block<false, true>(p, L, rho, w, Sg + (long)w * SS, Ek(w), lane, 64, wave_sync);
    wave_sync();
    if (p.ne && lane < S) {  // (factorize_w4's eliminated columns, unchanged)
        const int pe = p.eown[w * S + lane];
        if (pe >= 0) {
            const int e = pe - p.nb * S, ne2 = 2 * p.ne;
            const int2* __restrict__ et = (const int2*)p.etterm;
            double kjj = p.sigma, kpj = 0.0;
            for (int j = 0; j < p.eterm_max; ++j) {
                const int2 a = et[(long)j * ne2 + 2 * e], c = et[(long)j * ne2 + 2 * e + 1];
                kjj += a.y < 0 ? L.Pv[a.x] : rho_of(L.ct[a.y], rho) * L.Acsc[a.x & 0xFFFF] * L.Acsc[(unsigned)a.x >> 16];
                kpj += c.y < 0 ? L.Pv[c.x] : rho_of(L.ct[c.y], rho) * L.Acsc[c.x & 0xFFFF] * L.Acsc[(unsigned)c.x >> 16];
            }
            const double ed = 1.0 / kjj, ec = kpj * ed;
            oke = kjj > 0.0 && ed < __builtin_huge_val();
            Sg[(long)w * SS + lane * S + lane] -= kpj * ec;
            Fo[2 * e] = ec;
            Fo[2 * e + 1] = ed;
        }
        wave_sync();
    }
    bool okw = gj_seg<1, false, ROT>(Sg + (long)w * SS, bufw, w ? amax : 0, p.bsize[w], nullptr);
    okw = okw && __builtin_amdgcn_ballot_w64(!oke) == 0;
    __syncthreads();
#pragma unroll 1
    for (int k = 1; k < 4; ++k) {
        const double* Sp = Sg + (long)(k - 1) * SS;
        const double* E = Ek(k);
        double* const Gk = Gl + (long)(k * (k - 1) / 2 + k - 1) * gstride;  // G_{k,k-1} = -F_k
        const int l0 = p.toff[k - 1], bmax = p.bmax;
        for (int o = tid; o < as; o += TT) {
            const int r = o >> 5, j = o & (S - 1);
            double sacc = 0.0;
#pragma unroll 4
            for (int l = l0; l < l0 + bmax; ++l) sacc += E[r * S + l] * Sp[l * S + j];
            Gk[o] = -sacc;
        }
        __syncthreads();
        if (w == 0) {
            // the corner S_k = D_k - F_k E_k': -F_k E_k' = sum over G_{k,k-1} E_k'
            if (lane < amax * amax) {
                const int r = lane / amax, c = lane - r * amax;
                double sacc = 0.0;
#pragma unroll 4
                for (int l = l0; l < l0 + bmax; ++l) sacc += Gk[r * S + l] * E[c * S + l];
                dl[r * 16 + c] = sacc;
            }
            wave_sync();
            okw = gj_seg<2, false, ROT>(Sg + (long)k * SS, bufw, amax, p.bsize[k], dl) && okw;
        } else {
            // G_kj = -F_k G_{k-1,j} (j < k-1): G_{k,k-1} G_{k-1,j} for j < k-2, and
            // G_{k,k-1} G_{k-1,k-2} = F_k F_{k-1} for j = k-2
#pragma unroll 1
            for (int j = 0; j < k - 1; ++j) {
                const double* Gp = Gl + (long)((k - 1) * (k - 2) / 2 + j) * gstride;
                for (int o = tid - 64; o < as; o += TT - 64) {
                    const int r = o >> 5, c = o & (S - 1);
                    double sacc = 0.0;
#pragma unroll
                    for (int l = 0; l < 8; ++l)
                        if (l < amax) sacc += Gk[r * S + l] * Gp[l * S + c];
                    Gl[(long)(k * (k - 1) / 2 + j) * gstride + o] = sacc;
                }
            }
        }
        __syncthreads();
    }
    if (lane == 0) okf[w] = okw ? 1.0 : 0.0;
    __syncthreads();
    return okf[0] > 0.5 && okf[1] > 0.5 && okf[2] > 0.5 && okf[3] > 0.5;
}

__host__ __device__ inline double* w8_gpair(double* Fg, double* Hg, int amax, int q);  // (below)

// The eight-wave kernel's factorisation (solve_wave.hip::k_solve_w8, variant 18: mode 2,
// nb = 8, amax <= 12; TT = 512): factorize_w4 with eight blocks -- stage 1 pre-pivots all
// eight at once (wave k: block k), then the k = 1..7 chain: F_k = E_k S_{k-1}^{-1}
// (G_{k,k-1} = -F_k), wave 0 forms the corner and pivots it (gj_seg<2>, rolled: amax may
// exceed 8) while waves 1-7 form G_kj = -F_k G_{k-1,j}, j < k-1, reading G_{k-1,j} back
// from Hg (written by this workgroup one step earlier).  Outputs as factorize's mode 2;
// the tiles Sg lie in V past the scratch (w8_toff).
template <bool ROT = false, class KP>
__device__ __forceinline__ bool factorize_w8(const KP& p, SLds& L, const double rho, double* __restrict__ Fg,
                                             double* __restrict__ Hg, double* __restrict__ Sg) {
    constexpr int NB = 8, TT = 512;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int amax = p.amax, as = amax * S;
    double* const V = L.SP;
    double* const dl = V + (2 * NB - 1) * as;   // amax x amax, row stride 16
    double* const bufw = dl + 256 + w * 2 * S;  // the wave's Gauss-Jordan publish buffers
    double* const okf = dl + 256 + NB * 2 * S;
    auto Ek = [&](int k) __attribute__((always_inline)) { return V + k * as; };
    auto Fk = [&](int k) __attribute__((always_inline)) { return V + (NB - 1 + k) * as; };
    auto G = [&](int q) __attribute__((always_inline)) { return w8_gpair(Fg, Hg, amax, q); };
    auto wave_sync = []() __attribute__((always_inline)) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
#ifdef MPCQP_PHASE_PROF
    long long tf = clock64();
#define FPH(k) if (tid == 0) { const long long t_ = clock64(); L.pacc[k] += t_ - tf; tf = t_; }
#else
#define FPH(k)
#endif
    assemble_block<false, true>(p, L, rho, w, Sg + (long)w * SS, Ek(w), lane, 64, wave_sync);
    wave_sync();
    FPH(8)
    bool okw = gj_seg<1, false, ROT>(Sg + (long)w * SS, bufw, w ? amax : 0, p.bsize[w], nullptr);
    FPH(10)
    __syncthreads();
    FPH(11)
#pragma unroll 1
    for (int k = 1; k < NB; ++k) {
        const double* Sp = Sg + (long)(k - 1) * SS;
        const double* E = Ek(k);
        double* F = Fk(k);
        const int l0 = p.toff[k - 1], bmax = p.bmax;
        for (int o = tid; o < as; o += TT) {
            const int r = o >> 5, j = o & (S - 1);
            double sacc = 0.0;
#pragma unroll 4
            for (int l = l0; l < l0 + bmax; ++l) sacc += E[r * S + l] * Sp[l * S + j];
            F[o] = sacc;
            G(k * (k - 1) / 2 + k - 1)[o] = -sacc;
        }
        __syncthreads();
        FPH(9)
        if (w == 0) {
            for (int o = lane; o < amax * amax; o += 64) {  // S_k = D_k - F_k E_k' on the corner
                const int r = o / amax, c = o - r * amax;
                double sacc = 0.0;
#pragma unroll 4
                for (int l = l0; l < l0 + bmax; ++l) sacc += F[r * S + l] * E[c * S + l];
                dl[r * 16 + c] = -sacc;
            }
            wave_sync();
            okw = gj_seg<2, true>(Sg + (long)k * SS, bufw, amax, p.bsize[k], dl) && okw;
        } else {
#pragma unroll 1
            for (int j = 0; j < k - 1; ++j) {
                const bool adj = j == k - 2;
                const double* Gp = adj ? Fk(k - 1) : G((k - 1) * (k - 2) / 2 + j);
                const double sg = adj ? 1.0 : -1.0;
                for (int o = tid - 64; o < as; o += TT - 64) {
                    const int r = o >> 5, c = o & (S - 1);
                    double sacc = 0.0;
#pragma unroll 4
                    for (int l = 0; l < amax; ++l) sacc += F[r * S + l] * Gp[l * S + c];
                    G(k * (k - 1) / 2 + j)[o] = sg * sacc;
                }
            }
        }
        __syncthreads();
        FPH(11)
    }
    if (lane == 0) okf[w] = okw ? 1.0 : 0.0;
    __syncthreads();
    FPH(9)
#undef FPH
    bool ok = true;
#pragma unroll
    for (int k = 0; k < NB; ++k) ok = ok && okf[k] > 0.5;
    return ok;
}

// The 256-thread register-sweep kernels' factorisation (mode 1: F_k rows < amax and
// S_k^{-1} to the workspace; amax <= 16), split like factorize_w2 but on workspace
// tiles, since their LDS has no room for a tile per wave:
//   stage 1, the four waves in parallel: wave w takes blocks k = w, w + 4, ...: fills
//     D_k (zeros, the diagonal) and E_k in the workspace (Sg[k], Fg[k] rows < amax),
//     writes every target once, and pivots rows [a_k, 32) of D_k in place (gj_seg<1>,
//     a_0 = 0: block 0 whole);
//   then for k = 1..nb-1: F_k = E_k S_{k-1}^{-1} (over E_k's nonzero columns) -> LDS,
//     the corner correction -F_k E_k', F_k -> Fg[k] (waves 1-3) while wave 0 pivots
//     rows [0, amax) of S_k (gj_seg<2>).
// The Gauss-Jordan critical path is 32 + (nb - 1) amax pivot steps instead of 32 nb,
// and the assembly runs on four waves at once.  Same outputs as factorize's mode 1.
template <bool ROT = false, class KP>
__device__ __forceinline__ bool factorize_g(const KP& p, SLds& L, const double rho, double* __restrict__ Fg,
                                            double* __restrict__ Sg) {
    constexpr int TT = 256;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int nb = p.nb, amax = p.amax, as = amax * S;
    double* const V = L.SP;                    // LDS scratch (aliases the iteration vectors)
    double* const Fl = V;                      // F_k, amax x 32 (<= 512)
    double* const dl = V + 512;                // corner correction, row stride 16
    double* const bufw = V + 768 + w * 2 * S;  // the wave's Gauss-Jordan publish buffers
    double* const okf = V + 1024;
    auto gsync = []() __attribute__((always_inline)) {  // the wave's workspace stores before its loads
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    };
#ifdef MPCQP_PHASE_PROF
    long long tf = clock64();
#define FPH(k) if (tid == 0) { const long long t_ = clock64(); L.pacc[k] += t_ - tf; tf = t_; }
#else
#define FPH(k)
#endif
    bool okw = true;
#pragma unroll 1
    for (int k = w; k < nb; k += 4) {
        double* D = Sg + (long)k * SS;
        double* E = Fg + (long)k * SS;
        for (int e = 2 * lane; e < SS; e += 128) {
            const int r = e >> 5, c = e & (S - 1);  // c even: the diagonal is (r, r)
            const double dg = p.pad_var[k * S + r] >= 0 ? p.sigma : 1.0;
            *(double2*)(D + e) = make_double2(c == r ? dg : 0.0, c + 1 == r ? dg : 0.0);
        }
        for (int e = 2 * lane; e < as; e += 128) *(double2*)(E + e) = make_double2(0.0, 0.0);
        gsync();
        assemble_targets<false, false, true>(p, L, rho, k, D, E, lane, 64);
        gsync();
        FPH(8)
        okw = gj_seg<1, true>(D, bufw, k ? amax : 0, p.bsize[k], nullptr) && okw;
        FPH(10)
    }
    __syncthreads();
    FPH(11)
    const int bmax = p.bmax;
#pragma unroll 1
    for (int k = 1; k < nb; ++k) {
        const double* Sp = Sg + (long)(k - 1) * SS;
        const double* E = Fg + (long)k * SS;
        const int l0 = p.toff[k - 1];
        for (int o = tid; o < as; o += TT) {
            const int r = o >> 5, j = o & (S - 1);
            double sacc = 0.0;
#pragma unroll 4
            for (int l = l0; l < l0 + bmax; ++l) sacc += E[r * S + l] * Sp[l * S + j];
            Fl[o] = sacc;
        }
        __syncthreads();
        if (tid < amax * amax) {  // S_k = D_k - F_k E_k' on the corner
            const int r = tid / amax, c = tid - r * amax;
            double sacc = 0.0;
#pragma unroll 4
            for (int l = l0; l < l0 + bmax; ++l) sacc += Fl[r * S + l] * E[c * S + l];
            dl[r * 16 + c] = -sacc;
        }
        __syncthreads();
        FPH(9)
        if (w == 0) {
            okw = gj_seg<2, true>(Sg + (long)k * SS, bufw, amax, p.bsize[k], dl) && okw;
        } else {
            for (int o = tid - 64; o < as; o += TT - 64) Fg[(long)k * SS + o] = Fl[o];
        }
        __syncthreads();
        FPH(11)
    }
    if (lane == 0) okf[w] = okw ? 1.0 : 0.0;
    __syncthreads();
    FPH(9)
#undef FPH
    return okf[0] > 0.5 && okf[1] > 0.5 && okf[2] > 0.5 && okf[3] > 0.5;
}

// Assemble K's tiles for the current rho and factor them (block LDL'):
//   S_0 = D_0,  F_k = E_k S_{k-1}^{-1},  S_k = D_k - F_k E_k',  H_{k-1} = F_k'
// E_k is nonzero only in its first amax rows (block k's first BFS level), so F_k
// has amax nonzero rows and F_k E_k' touches only the leading amax x amax corner
// of S_k.  F_k, H_k, S_k^{-1} go to the per-instance workspace (Fg, Hg, Sg); their
// entries outside those rows / columns are never written (zero from allocation).
// S_k^{-1} by Gauss-Jordan (SPD: no pivoting) on register-resident tile elements.
// What else is stored depends on the solve variant (KParams::mode):
//   0: F_k and H_k = F_k' as full tiles (solves reading the tiles from the workspace)
//   1: F_k only (register sweep; H is loaded as F transposed)
//   2: the blocks of L^{-1}:  G_kj = (-1)^{k-j} F_k F_{k-1} .. F_{j+1}  (j < k), amax x 32
//      each, in Hg at pair (k, j) -> k(k-1)/2 + j, row stride 32 (three-phase solve).
// Returns false on a non-positive pivot (OSQP: "problem non convex").
// POL: the polish system P + delta I + A' diag(w) A instead (solve.hip::k_polish): row
// weights w_i = (number of active copies of row i, from ct bits 0/1) * rho with
// rho = 1 / delta, diagonal delta, factor stored as in mode 1.
template <int TT, class KP, bool POL = false, bool ROT = false>
__device__ __forceinline__ bool factorize(const KP& p, SLds& L, double rho, double* __restrict__ Fg,
                                          double* __restrict__ Hg, double* __restrict__ Sg) {
    if constexpr (TT == 128 && !POL) {  // the two-wave kernel (variant 10: nb = 4, amax <= 8)
        if (p.mode == 2 && p.nb == 4 && p.amax <= 8) return factorize_w2<ROT>(p, L, rho, Hg, Sg);
    }
    if constexpr (TT == 256 && !POL) {  // the register-sweep kernels (variants 1-3), the four-wave kernel (17)
        if (p.mode == 1 && p.amax <= 16) return factorize_g<ROT>(p, L, rho, Fg, Sg);
        if (p.variant == 17 && p.mode == 2 && p.nb == 4 && p.amax <= 8) return factorize_w4<ROT>(p, L, rho, Hg, Sg, Fg);
    }
    if constexpr (TT == 512 && !POL) {  // the eight-wave kernel (18)
        if (p.variant == 18 && p.mode == 2 && p.nb == 8 && p.amax <= 12) return factorize_w8<ROT>(p, L, rho, Fg, Hg, Sg);
    }
    const int tid = threadIdx.x;
    const int nb = p.nb, amax = p.amax, mode = POL ? 1 : p.mode;
    const long gstride = (long)amax * S;
    bool ok = true;
    double* SP = L.SP;
    double* DK = L.DK;
    double* EK = L.EK;
#ifdef MPCQP_PHASE_PROF
    long long tf = clock64();
#define FPH(k) if (tid == 0) { const long long t_ = clock64(); L.pacc[k] += t_ - tf; tf = t_; }
#else
#define FPH(k)
#endif
    auto assemble = [&](const int k, double* __restrict__ D, double* __restrict__ E, const int t0, const int nt,
                        auto sync) __attribute__((always_inline)) {
        assemble_block<POL, false>(p, L, rho, k, D, E, t0, nt, sync);
    };
    auto block_sync = []() __attribute__((always_inline)) { __syncthreads(); };
    auto wave_sync = []() __attribute__((always_inline)) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    // OVL (two waves, E_k within half a tile): while wave 0 inverts S_k, wave 1 assembles
    // D_{k+1} into SP (dead once F_k's products are done) and E_{k+1} into the other half
    // of the E tile; the half holding E_k (dead as well) is the Gauss-Jordan buffer.
    const bool OVL = TT == 128 && !POL && amax * S <= SS / 2;
    auto Eh = [&](int k) __attribute__((always_inline)) { return OVL ? EK + (k & 1) * (SS / 2) : EK; };
    if (OVL) {
        assemble(0, DK, Eh(0), tid, TT, block_sync);
        __syncthreads();
    }
#pragma unroll 1
    for (int k = 0; k < nb; ++k) {
        double* const Ek = Eh(k);
        if (!OVL) {
            assemble(k, DK, EK, tid, TT, block_sync);
            __syncthreads();
        }
        FPH(8)
        if (k > 0) {
            // F_k = E_k S_{k-1}^{-1} (rows < amax), then written over S_{k-1}^{-1}'s tile
            constexpr int NF = SS / TT;  // per-thread F buffer (dynamically indexed)
            double f[NF];
            int nf = 0;
#pragma unroll 1
            for (int o = tid; o < amax * S; o += TT, ++nf) {
                const int r = o >> 5, j = o & (S - 1);
                double sacc = 0.0;
#pragma unroll 8
                for (int l = 0; l < S; ++l) sacc += Ek[r * S + l] * SP[l * S + j];
                f[nf & (NF - 1)] = sacc;
                if (mode < 2) Fg[(long)k * SS + r * S + j] = sacc;
                if (mode == 0) Hg[(long)(k - 1) * SS + j * S + r] = sacc;
                if (mode == 2) Hg[(long)(k * (k - 1) / 2 + k - 1) * gstride + o] = -sacc;
            }
            __syncthreads();  // every read of S_{k-1}^{-1} done
            nf = 0;
#pragma unroll 1
            for (int o = tid; o < amax * S; o += TT, ++nf) SP[o] = f[nf & (NF - 1)];
            __syncthreads();
            if (mode == 2) {  // G_kj = -F_k G_{k-1,j} (G_{k-1,j} has amax nonzero rows)
#pragma unroll 1
                for (int j = 0; j < k - 1; ++j) {
                    const double* Gp = Hg + (long)((k - 1) * (k - 2) / 2 + j) * gstride;
                    double* Gk = Hg + (long)(k * (k - 1) / 2 + j) * gstride;
#pragma unroll 1
                    for (int o = tid; o < amax * S; o += TT) {
                        const int r = o >> 5, c = o & (S - 1);
                        double sacc = 0.0;
                        if constexpr (TT == 128) {
                            // two-wave kernel (mode 2 there has amax <= 8, variant_fits): the 8
                            // loads of G_{k-1,j} (global, just written) go out together; rows >=
                            // amax stay inside the tile array.  Not in the 256-thread kernels:
                            // the unrolled loads raise factorize_nl's SGPR use, which costs the
                            // calling solve loop SGPR spills (cfg 3 solve +6 %).
                            double gv[8];
#pragma unroll
                            for (int l = 0; l < 8; ++l) gv[l] = Gp[l * S + c];
#pragma unroll
                            for (int l = 0; l < 8; ++l)
                                if (l < amax) sacc += SP[r * S + l] * gv[l];
                        } else {
#pragma unroll 1
                            for (int l = 0; l < amax; ++l) sacc += SP[r * S + l] * Gp[l * S + c];
                        }
                        Gk[o] = -sacc;
                    }
                }
            }
            // S_k = D_k - F_k E_k' on the leading amax x amax corner
#pragma unroll 1
            for (int o = tid; o < amax * amax; o += TT) {
                const int r = o / amax, c = o - r * amax;
                double sacc = 0.0;
#pragma unroll 8
                for (int l = 0; l < S; ++l) sacc += SP[r * S + l] * Ek[c * S + l];
                DK[r * S + c] -= sacc;
            }
            __syncthreads();
        }
        FPH(9)
        {
            // one wave inverts the tile (no barrier per pivot); the verdict goes through LDS
            double* okslot = Ek + 2 * S;
            if (tid < 64) {
                const bool okw = gj_wave<(TT > 128)>(DK, Ek, Sg + (long)k * SS, p.bsize[k]);
                if (tid == 0) okslot[0] = okw ? 1.0 : 0.0;
            } else if (OVL && tid < 128 && k + 1 < nb) {
                assemble(k + 1, SP, Eh(k + 1), tid - 64, 64, wave_sync);
            }
            __syncthreads();
            if (!(okslot[0] > 0.5)) ok = false;
            FPH(10)
        }
        double* t = SP; SP = DK; DK = t;  // S_k^{-1} becomes "previous" (OVL: D_{k+1} is in DK now)
        if (!OVL) __syncthreads();
        FPH(11)
    }
#undef FPH
    return ok;
}

// Gather list of one column (A' w) or row (A x) of A: K packed entries
// (value position in the padded-CSC copy of A in LDS | vector index << 16), padded
// with the zero slot Acsc[nnzA] -- no per-entry branches, all 2K LDS reads in flight.
template <int K>
struct Gather {
    unsigned e[K];
    // list[k * stride].  `stride` is read through a volatile pointer (a scalar load at
    // every run start), so the k * stride offsets cannot be hoisted out of the solve loop
    // and held in registers for its whole length (measured: 28 more VGPR spills in the
    // 256-thread nb = 8 kernel when they are).
    __device__ __forceinline__ void load(const int* list, const volatile int* stride) {
        const int st = *stride;
#pragma unroll
        for (int k = 0; k < K; ++k) e[k] = (unsigned)list[k * st];
    }
    __device__ __forceinline__ void clear(int zero_pos) {
#pragma unroll
        for (int k = 0; k < K; ++k) e[k] = (unsigned)zero_pos;
    }
    // an opaque zero offset keeps the LDS addresses from being hoisted into
    // registers across the ADMM loop
    __device__ __forceinline__ double dot(const double* A, const double* vec) const {
        int opq = 0;
        asm volatile("" : "+s"(opq));
        double t[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const unsigned ek = e[k] + (unsigned)opq;  // unpacked inside the loop: the packed
            t[k] = A[ek & 0xFFFFu] * vec[ek >> 16];    // word is the only register it costs
        }
#pragma unroll
        for (int w = 1; w < K; w *= 2)
#pragma unroll
            for (int k = 0; k + w < K; k += 2 * w) t[k] += t[k + w];
        return t[0];
    }
};

// Gather with both halves of an entry as double offsets from the dynamic LDS base (the
// A value's and the vector element's), so a dot product forms its addresses from the entry
// alone -- no base pointer (kept in a spilled SGPR by the long-horizon kernel) reloaded in
// front of its reads.  oA / oV: the A values' and the vector's offsets from the base
// (< 65536 doubles: LDS holds at most 20 K).
template <int K>
struct GatherR {
    unsigned e[K];
    __device__ __forceinline__ void load(const int* list, const volatile int* stride, unsigned oA, unsigned oV) {
        const int st = *stride;
        const unsigned o = oA + (oV << 16);
#pragma unroll
        for (int k = 0; k < K; ++k) e[k] = (unsigned)list[k * st] + o;
    }
    __device__ __forceinline__ void load(const int* list, int st, unsigned oA, unsigned oV) {
        const unsigned o = oA + (oV << 16);
#pragma unroll
        for (int k = 0; k < K; ++k) e[k] = (unsigned)list[k * st] + o;
    }
    __device__ __forceinline__ void clear(int zero_pos, unsigned oA, unsigned oV) {
#pragma unroll
        for (int k = 0; k < K; ++k) e[k] = (unsigned)zero_pos + oA + (oV << 16);
    }
    __device__ __forceinline__ double dot() const {
        extern __shared__ __attribute__((aligned(16))) double sm[];
        int opq = 0;
        asm volatile("" : "+s"(opq));  // (Gather::dot: the unpacked addresses are not hoisted out of the loop)
        double t[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const unsigned ek = e[k] + (unsigned)opq;
            t[k] = sm[ek & 0xFFFFu] * sm[ek >> 16];
        }
#pragma unroll
        for (int w = 1; w < K; w *= 2)
#pragma unroll
            for (int k = 0; k + w < K; k += 2 * w) t[k] += t[k + w];
        return t[0];
    }
};

struct Res {  // update_info results
    double pri, dua, nz, nax, nq, naty, npx;    // termination (unscaled)
    double rpri, rdua, rz, rax, rq, raty, rpx;  // rho estimate (scaled space)
    __device__ __forceinline__ void save(double* d) const {
        d[0] = pri; d[1] = dua; d[2] = nz; d[3] = nax; d[4] = nq; d[5] = naty; d[6] = npx;
        d[7] = rpri; d[8] = rdua; d[9] = rz; d[10] = rax; d[11] = rq; d[12] = raty; d[13] = rpx;
    }
    __device__ __forceinline__ void restore(const double* d) {
        pri = d[0]; dua = d[1]; nz = d[2]; nax = d[3]; nq = d[4]; naty = d[5]; npx = d[6];
        rpri = d[7]; rdua = d[8]; rz = d[9]; rax = d[10]; rq = d[11]; raty = d[12]; rpx = d[13];
    }
};

// LDS carve of the solve kernel (doubles unless noted):
//   Acsc[nnzA+1] Pv[nnzP+1] lo[mp] up[mp] qv[npad] X[npad] Z[mp]   (mp = m rounded up to 64)
//   V = max(3 S*S, w[mp] rb[npad] xt[npad] ys[mp] dY[mp] gl[...])   (factor scratch aliases the vectors;
//       ys is saved to the workspace around a refactorisation)
//   red[128] res[16] pacc[16] cor[nb*S] tv[npad] ct[mp bytes] flag
// rb holds delta_x and dY delta_y of the last iteration after its update phase;
// ys holds y whenever the out-of-line phases run.
// V holds the per-iteration vectors, then (mode 2) an LDS copy of the G blocks for
// the wave kernel; the factorisation's three scratch tiles alias all of it.
__host__ __device__ inline long solve_glen(int nb, int amax, int mode) {
    // rows padded to >= 8 (nb = 4) or to 12 (nb = 8, the eight-wave kernel), + a zero pair
    return mode == 2 ? ((long)nb * (nb - 1) / 2 + 1) * (nb > 4 ? 12 : (amax > 8 ? amax : 8)) * S : 0;
}
// The eight-wave kernel (variant 18: mode 2, nb = 8, amax <= 12) keeps everything in V:
// its factorisation scratch at [0, w8_toff), the S_k^{-1} tiles after it, and its
// reduction buffer (256) at w8_roff.  The G copy (at 3 mp + 2 npad) overlaps the tiles:
// it is filled once the tiles are in registers (solve_wave.hip::solve_w8_body).
__host__ __device__ inline long w8_toff(int amax) { return (15L * amax * S + 256 + 16 * S + 64 + 63) & ~63L; }
// pair q's G block (amax x 32) of one instance: the 28 pairs outgrow the instance's
// H tiles (nb SS doubles) for amax > 9 and continue in its F tiles (unused in mode 2)
__host__ __device__ inline double* w8_gpair(double* Fg, double* Hg, int amax, int q) {
    const int gs = amax * S, nqh = 8 * SS / gs;
    return q < nqh ? Hg + (long)q * gs : Fg + (long)(q - nqh) * gs;
}
__host__ __device__ inline long w8_roff(int m, int npad, int amax) {
    const long t = w8_toff(amax) + 8L * SS, g = 3L * ((m + 63) & ~63) + 2L * npad + solve_glen(8, amax, 2);
    return t > g ? t : g;
}
// row arrays are padded to whole waves (the wave kernel's rows i = lane + 64 s are
// then all in range; padded rows are inert: l = u = 0, empty gather list)
__host__ __device__ inline int solve_mpad(int m) { return (m + 63) & ~63; }
__host__ __device__ inline long solve_vlen(int m, int npad, int nb, int amax, int mode) {
    const long a = 3L * solve_mpad(m) + 2L * npad + solve_glen(nb, amax, mode), b = 3L * SS;
    if (mode == 2 && nb > 4) {
        const long c = w8_roff(m, npad, amax) + 256;
        return c > a ? c : a;
    }
    return a > b ? a : b;
}

struct SL2 {  // full carve (SLds + the solve-kernel-only arrays)
    SLds L;
    double *X, *Z, *dY;
};

// every array starts on a 16-byte boundary (the wave kernels' broadcast reads are
// ds_read_b128); A16 tells the compiler so
__host__ __device__ inline long al2(long x) { return (x + 1) & ~1L; }
#define A16(ptr) ((double*)__builtin_assume_aligned((ptr), 16))

// bytes of the carve below (what lds_solve_bytes reports)
template <class KP>
__host__ __device__ inline size_t lds_base_bytes(const KP& p) {
    const size_t mp = (size_t)solve_mpad(p.m);
    return sizeof(double) * ((size_t)al2(p.nnzA + 1) + (size_t)al2(p.nnzP + 1) + 3 * mp + 2 * (size_t)p.npad +
                             (size_t)solve_vlen(p.m, p.npad, p.nb, p.amax, p.mode) + 160 + (size_t)p.nb * S +
                             (size_t)p.npad) +
           mp + 64;
}

template <class KP>
__device__ __forceinline__ SL2 carve(const KP& p) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    SL2 c;
    const int mp = solve_mpad(p.m), npad = p.npad;
    c.L.Acsc = A16(sm);
    c.L.Pv = A16(c.L.Acsc + al2(p.nnzA + 1));  // Acsc[nnzA] = 0: gather padding
    c.L.lo = A16(c.L.Pv + al2(p.nnzP + 1));    // Pv[nnzP] = 0: P-list padding
    c.L.up = A16(c.L.lo + mp);
    c.L.qv = A16(c.L.up + mp);
    c.X = A16(c.L.qv + npad);
    c.Z = A16(c.X + npad);
    double* V = A16(c.Z + mp);
    c.L.w = V;
    c.L.rb = A16(c.L.w + mp);
    c.L.xt = A16(c.L.rb + npad);
    c.L.ys = A16(c.L.xt + npad);
    c.dY = A16(c.L.ys + mp);
    c.L.SP = V;
    c.L.EK = A16(c.L.SP + SS);
    c.L.DK = A16(c.L.EK + SS);
    c.L.gl = A16(c.dY + mp);
    c.L.red = A16(V + solve_vlen(p.m, npad, p.nb, p.amax, p.mode));
    c.L.res = A16(c.L.red + 128);
    c.L.pacc = (long long*)(c.L.res + 16);
    c.L.cor = A16((double*)(c.L.pacc + 16));
    c.L.dx = p.mode == 2 ? c.L.xt : c.L.rb;
    c.L.tv = A16(c.L.cor + p.nb * S);
    c.L.ct = (signed char*)(c.L.tv + npad);
    c.L.flag = (int*)(c.L.ct + mp);
    return c;
}

// EDL (the one-shot fused kernel's form 2, one_shot_form): the setup leaves E and D in the carve's
// V span after gl (free in the four-wave kernel: its V is sized for 3 S x S of scratch) instead of
// in the workspace; the checks and finalize read them there
template <class KP>
__device__ __forceinline__ double* edl_E(const KP& p, const SL2& c) {
    return A16(c.L.gl + solve_glen(p.nb, p.amax, p.mode));
}
template <class KP>
__device__ __forceinline__ double* edl_D(const KP& p, const SL2& c) {
    return A16(edl_E(p, c) + al2(p.m));
}

// LDS scalar slots (in res[14..15] and flag[1..]): shared outcome of the out-of-line phases
struct Shared {
    double* res;  // [0..13] Res, [14] obj, [15] new rho
    int* flag;    // [0] scratch, [1] status, [2] dx_scaled, [3] dy_scaled
};

// status "non convex" of an early exit (invalid data, first factorisation failed), with
// the per-call copies mpcqp_solve_device asks for
// (no ADMM iteration ran: the iteration count is 0, not the previous solve's, which
// k_order would otherwise take for a long solve)
template <class KP>
__device__ __forceinline__ void fail_status(const KP& p, long b) {
    p.status[b] = MPCQP_NON_CVX_;
    p.iter[b] = 0;
    if (p.ostat) p.ostat[b] = MPCQP_NON_CVX_;
    if (p.oiter) p.oiter[b] = 0;
}

// ---- out-of-line phases: everything they need is in LDS or in the plan ----
// dot of a packed gather list (value index | vector index << 16) with cnt entries
__device__ __forceinline__ double list_dot(const int* __restrict__ list, int stride, int cnt, const double* V,
                                           const double* v) {
    double acc = 0.0;
#pragma unroll 4
    for (int k = 0; k < cnt; ++k) {
        const unsigned e = (unsigned)list[(long)k * stride];
        acc += V[e & 0xFFFFu] * v[e >> 16];
    }
    return acc;
}
template <class KP>
__device__ __forceinline__ double row_dot(const KP& p, const double* A, const double* v, int i) {
    return list_dot(p.grow + i, p.m, p.gk, A, v);
}
template <class KP>
__device__ __forceinline__ double col_dot(const KP& p, const double* A, const double* v, int pc) {
    return list_dot(p.gcol + pc, p.npad, p.gk, A, v);
}
template <class KP>
__device__ __forceinline__ double psym_dot(const KP& p, const double* Pv, const double* v, int pc) {
    return list_dot(p.gpsym + pc, p.npad, p.pk, Pv, v);
}

// update_info: residuals and the norms of their tolerances (OSQP compute_pri_res /
// compute_dua_res / compute_pri_tol / compute_dua_tol, scaled and unscaled)
template <int TT, bool EDL = false>
__device__ __forceinline__ void update_info_ph(const KParams* gp, long b, double cinv) {
    KPc& p = kconst(gp);
    SL2 c = carve(p);
    const int tid = threadIdx.x, m = p.m, npad = p.npad;
    const double* Eg = EDL ? edl_E(p, c) : p.E + b * m;
    const double* Dg = EDL ? edl_D(p, c) : p.D + b * npad;
    double v[14];
#pragma unroll
    for (int k = 0; k < 14; ++k) v[k] = 0.0;
#pragma unroll 1
    for (int i = tid; i < m; i += TT) {
        const double ax = row_dot(p, c.L.Acsc, c.X, i);
        const double zi = c.Z[i];
        const double pr = ax - zi;
        const double ei = 1.0 / Eg[i];
        v[0] = cmax(v[0], fabs(ei * pr));
        v[2] = cmax(v[2], fabs(ei * zi));
        v[3] = cmax(v[3], fabs(ei * ax));
        v[7] = cmax(v[7], fabs(pr));
        v[9] = cmax(v[9], fabs(zi));
        v[10] = cmax(v[10], fabs(ax));
    }
#pragma unroll 1
    for (int pc = tid; pc < npad; pc += TT) {
        if (p.pad_var[pc] < 0) continue;
        const double px = psym_dot(p, c.L.Pv, c.X, pc);
        const double aty = col_dot(p, c.L.Acsc, c.L.ys, pc);
        const double q = c.L.qv[pc];
        const double d = (q + px) + aty;
        const double di = 1.0 / Dg[pc];
        v[1] = cmax(v[1], fabs(di * d));
        v[4] = cmax(v[4], fabs(di * q));
        v[5] = cmax(v[5], fabs(di * aty));
        v[6] = cmax(v[6], fabs(di * px));
        v[8] = cmax(v[8], fabs(d));
        v[11] = cmax(v[11], fabs(q));
        v[12] = cmax(v[12], fabs(aty));
        v[13] = cmax(v[13], fabs(px));
    }
    double* r = c.L.red + (TT / 64 * 14 <= 64 ? 64 : 112);  // after the per-wave maxima
    block_max_to<TT>(v, c.L.red, r);
    if (tid == 0) {
        Res R;
        if (p.scaling && !p.scaled_term) {
            R.pri = r[0]; R.dua = cinv * r[1];
            R.nz = r[2]; R.nax = r[3]; R.nq = r[4]; R.naty = r[5]; R.npx = r[6];
        } else {
            R.pri = r[7]; R.dua = r[8];
            R.nz = r[9]; R.nax = r[10]; R.nq = r[11]; R.naty = r[12]; R.npx = r[13];
        }
        R.rpri = r[7]; R.rdua = r[8]; R.rz = r[9]; R.rax = r[10]; R.rq = r[11]; R.raty = r[12]; R.rpx = r[13];
        if (m == 0) R.pri = 0.0;
        R.save(c.L.res);
    }
    __syncthreads();
}
template <int TT, bool EDL = false>
__device__ __noinline__ void update_info_nl(const KParams* gp, long b, double cinv) {
    update_info_ph<TT, EDL>(gp, b, cinv);
}

// is_primal_infeasible (delta_y in dY, projected in place as OSQP does)
template <int TT, bool EDL = false, class KP>
__device__ bool primal_infeasible(const KP& p, SL2& c, long b, double eps) {
    const int tid = threadIdx.x, m = p.m, npad = p.npad;
    const bool unscale = p.scaling && !p.scaled_term;
    const double* Eg = EDL ? edl_E(p, c) : p.E + b * m;
    const double* Dg = EDL ? edl_D(p, c) : p.D + b * npad;
    double nd[1] = {0.0};
#pragma unroll 1
    for (int i = tid; i < m; i += TT) {
        double d = c.dY[i];
        if (c.L.up[i] > OSQP_INFTY * MIN_SCALING) d = (c.L.lo[i] < -OSQP_INFTY * MIN_SCALING) ? 0.0 : cmin(d, 0.0);
        else if (c.L.lo[i] < -OSQP_INFTY * MIN_SCALING) d = cmax(d, 0.0);
        c.dY[i] = d;
        nd[0] = cmax(nd[0], fabs(unscale ? Eg[i] * d : d));
    }
    block_max<TT>(nd, c.L.red);
    const double norm_dy = nd[0];
    if (!(norm_dy > eps)) return false;
    double sum[1] = {0.0};
#pragma unroll 1
    for (int i = tid; i < m; i += TT) sum[0] += c.L.up[i] * cmax(c.dY[i], 0.0) + c.L.lo[i] * cmin(c.dY[i], 0.0);
    block_sum<TT>(sum, c.L.red);
    if (!(sum[0] < eps * norm_dy)) return false;
    double na[1] = {0.0};
#pragma unroll 1
    for (int pc = tid; pc < npad; pc += TT) {
        if (p.pad_var[pc] < 0) continue;
        double a = col_dot(p, c.L.Acsc, c.dY, pc);
        if (unscale) a *= 1.0 / Dg[pc];
        na[0] = cmax(na[0], fabs(a));
    }
    block_max<TT>(na, c.L.red);
    return na[0] < eps * norm_dy;
}

// is_dual_infeasible (delta_x in dx)
template <int TT, bool EDL = false, class KP>
__device__ bool dual_infeasible(const KP& p, SL2& c, long b, double cs_, double eps) {
    const int tid = threadIdx.x, m = p.m, npad = p.npad;
    const bool unscale = p.scaling && !p.scaled_term;
    const double* Eg = EDL ? edl_E(p, c) : p.E + b * m;
    const double* Dg = EDL ? edl_D(p, c) : p.D + b * npad;
    const double cs = unscale ? cs_ : 1.0;
    double v[1] = {0.0}, sum[1] = {0.0};
#pragma unroll 1
    for (int pc = tid; pc < npad; pc += TT) {
        if (p.pad_var[pc] < 0) continue;
        const double dx = c.L.dx[pc];
        v[0] = cmax(v[0], fabs(unscale ? Dg[pc] * dx : dx));
        sum[0] += c.L.qv[pc] * dx;
    }
    block_max<TT>(v, c.L.red);
    const double norm_dx = v[0];
    if (!(norm_dx > eps)) return false;
    block_sum<TT>(sum, c.L.red);
    if (!(sum[0] < cs * eps * norm_dx)) return false;
    double np[1] = {0.0};
#pragma unroll 1
    for (int pc = tid; pc < npad; pc += TT) {
        if (p.pad_var[pc] < 0) continue;
        double a = psym_dot(p, c.L.Pv, c.L.dx, pc);
        if (unscale) a *= 1.0 / Dg[pc];
        np[0] = cmax(np[0], fabs(a));
    }
    block_max<TT>(np, c.L.red);
    if (!(np[0] < cs * eps * norm_dx)) return false;
    bool viol = false;
#pragma unroll 1
    for (int i = tid; i < m; i += TT) {
        double a = row_dot(p, c.L.Acsc, c.L.dx, i);
        if (unscale) a *= 1.0 / Eg[i];
        if ((c.L.up[i] < OSQP_INFTY * MIN_SCALING && a > eps * norm_dx) ||
            (c.L.lo[i] > -OSQP_INFTY * MIN_SCALING && a < -eps * norm_dx))
            viol = true;
    }
    return !block_any<TT>(viol, c.L.flag);
}

// check_termination on the Res in LDS; status / obj / certificate flags in LDS.
template <int TT, bool EDL = false>
__device__ __forceinline__ int check_termination_ph(const KParams* gp, long b, double cval, double cinv,
                                                 int approximate) {
    KPc& p = kconst(gp);
    SL2 c = carve(p);
    Res R;
    R.restore(c.L.res);
    double eps_abs = p.eps_abs, eps_rel = p.eps_rel, eps_pinf = p.eps_pinf, eps_dinf = p.eps_dinf;
    int st = MPCQP_UNSOLVED_;
    double obj = c.L.res[14];
    bool done = false;
    if (R.pri > OSQP_INFTY || R.dua > OSQP_INFTY) {
        st = MPCQP_NON_CVX_;
        obj = __builtin_nan("");
        done = true;
    } else {
        if (approximate) { eps_abs *= 10; eps_rel *= 10; eps_pinf *= 10; eps_dinf *= 10; }
        bool prim_ok = false, dual_ok = false, prim_inf = false, dual_inf = false;
        const bool unscale = p.scaling && !p.scaled_term;
        if (p.m == 0) prim_ok = true;
        else {
            const double ep = eps_abs + eps_rel * cmax(R.nz, R.nax);
            if (R.pri < ep) prim_ok = true;
            else prim_inf = primal_infeasible<TT, EDL>(p, c, b, eps_pinf);
        }
        double mx = cmax(cmax(R.nq, R.naty), R.npx);
        if (unscale) mx *= cinv;
        if (R.dua < eps_abs + eps_rel * mx) dual_ok = true;
        else dual_inf = dual_infeasible<TT, EDL>(p, c, b, cval, eps_dinf);
        if (prim_ok && dual_ok) {
            st = approximate ? MPCQP_SOLVED_INACCURATE_ : MPCQP_SOLVED_;
            done = true;
        } else if (prim_inf) {
            st = approximate ? MPCQP_PRIMAL_INFEASIBLE_INACCURATE_ : MPCQP_PRIMAL_INFEASIBLE_;
            obj = OSQP_INFTY;
            if (threadIdx.x == 0) c.L.flag[3] = unscale;
            done = true;
        } else if (dual_inf) {
            st = approximate ? MPCQP_DUAL_INFEASIBLE_INACCURATE_ : MPCQP_DUAL_INFEASIBLE_;
            obj = -OSQP_INFTY;
            if (threadIdx.x == 0) c.L.flag[2] = unscale;
            done = true;
        }
    }
    __syncthreads();
    if (done && threadIdx.x == 0) { c.L.flag[1] = st; c.L.res[14] = obj; }
    __syncthreads();
    return done ? st : MPCQP_UNSOLVED_;
}
template <int TT, bool EDL = false>
__device__ __noinline__ int check_termination_nl(const KParams* gp, long b, double cval, double cinv,
                                                 int approximate) {
    return check_termination_ph<TT, EDL>(gp, b, cval, cinv, approximate);
}

// compute_obj_val (needs X)
template <int TT>
__device__ __forceinline__ void objective_ph(const KParams* gp, double cinv) {
    KPc& p = kconst(gp);
    SL2 c = carve(p);
    const int tid = threadIdx.x;
    double sacc[1] = {0.0};
#pragma unroll 1
    for (int v = tid; v < p.nnzP; v += TT) {
        const int r = p.p_r[v], cc = p.p_c[v];
        sacc[0] += (r == cc) ? 0.5 * c.L.Pv[v] * c.X[r] * c.X[r] : c.L.Pv[v] * c.X[r] * c.X[cc];
    }
#pragma unroll 1
    for (int pc = tid; pc < p.npad; pc += TT) sacc[0] += c.L.qv[pc] * c.X[pc];
    block_sum<TT>(sacc, c.L.red);
    if (tid == 0) c.L.res[14] = p.scaling ? sacc[0] * cinv : sacc[0];
    __syncthreads();
}
template <int TT>
__device__ __noinline__ void objective_nl(const KParams* gp, double cinv) {
    objective_ph<TT>(gp, cinv);
}

// store_solution + info (y is in ys).  ONE (the one-shot fused setup + solve, mpcqp_set_one_shot):
// no later call reads the workspace, so the warm-start iterates x, z, y and the infeasibility
// certificates are not stored -- the outputs, the status / iteration count (the next dispatch
// order) and the info are
template <int TT, bool ONE = false, bool EDL = false>
__device__ __forceinline__ void finalize_ph(const KParams* gp, long b, double* __restrict__ xo,
                                         double* __restrict__ yo, double cinv, double rho, int status,
                                         int info_iter, int rho_updates, int* ostat, int* oiter) {
    KPc& p = kconst(gp);
    SL2 c = carve(p);
    const int tid = threadIdx.x, n = p.n, m = p.m, npad = p.npad;
    const double* Eg = EDL ? edl_E(p, c) : p.E + b * m;
    const double* Dg = EDL ? edl_D(p, c) : p.D + b * npad;
    Res R;
    R.restore(c.L.res);
    double rho_est;
    {
        const double pr = R.rpri / (cmax(R.rz, R.rax) + DIVISION_TOL);
        const double du = R.rdua / (cmax(cmax(R.rq, R.raty), R.rpx) + DIVISION_TOL);
        rho_est = cmin(cmax(rho * sqrt(pr / (du + DIVISION_TOL)), RHO_MIN), RHO_MAX);
    }
    const bool has_sol = !(status == MPCQP_PRIMAL_INFEASIBLE_ || status == MPCQP_PRIMAL_INFEASIBLE_INACCURATE_ ||
                           status == MPCQP_DUAL_INFEASIBLE_ || status == MPCQP_DUAL_INFEASIBLE_INACCURATE_ ||
                           status == MPCQP_NON_CVX_);
    const bool pinf = status == MPCQP_PRIMAL_INFEASIBLE_ || status == MPCQP_PRIMAL_INFEASIBLE_INACCURATE_;
    const bool dinf = status == MPCQP_DUAL_INFEASIBLE_ || status == MPCQP_DUAL_INFEASIBLE_INACCURATE_;
    // the objective: computed (objective_nl) when there is a solution, else the value the
    // status implies (OSQP: +inf primal infeasible, -inf dual infeasible, NaN non-convex)
    const double obj = has_sol ? c.L.res[14] : (pinf ? OSQP_INFTY : (dinf ? -OSQP_INFTY : __builtin_nan("")));
    const bool dx_scaled = c.L.flag[2] != 0, dy_scaled = c.L.flag[3] != 0;
    double nrm[2] = {0.0, 0.0};
#pragma unroll 1
    for (int pc = tid; pc < npad; pc += TT) {
        double dx = c.L.dx[pc];
        if (dx_scaled) dx *= Dg[pc];
        c.L.dx[pc] = dx;
        nrm[1] = cmax(nrm[1], fabs(dx));
    }
#pragma unroll 1
    for (int i = tid; i < m; i += TT) {
        double dy = c.dY[i];
        if (dy_scaled) dy *= Eg[i];
        c.dY[i] = dy;
        nrm[0] = cmax(nrm[0], fabs(dy));
    }
    block_max<TT>(nrm, c.L.red);
#pragma unroll 1
    for (int pc = tid; pc < npad; pc += TT) {
        const int j = p.pad_var[pc];
        const double xv = c.X[pc];
        if (j >= 0) {
            if (xo) xo[b * n + j] = has_sol ? (p.scaling ? Dg[pc] * xv : xv) : __builtin_nan("");
            if (!ONE) p.dxc[b * n + j] = dinf ? c.L.dx[pc] * (1.0 / nrm[1]) : c.L.dx[pc];
        }
        if (!ONE) p.x[b * npad + pc] = has_sol ? xv : 0.0;
    }
#pragma unroll 1
    for (int i = tid; i < m; i += TT) {
        const double yv = c.L.ys[i];
        if (yo) yo[b * m + i] = has_sol ? (p.scaling ? (Eg[i] * yv) * cinv : yv) : __builtin_nan("");
        if (!ONE) {
            p.dyc[b * m + i] = pinf ? c.dY[i] * (1.0 / nrm[0]) : c.dY[i];
            p.y[b * m + i] = has_sol ? yv : 0.0;
            p.z[b * m + i] = has_sol ? c.Z[i] : 0.0;
        }
    }
    if (tid == 0) {
        p.status[b] = status;
        p.iter[b] = info_iter;
        if (ostat) ostat[b] = status;
        if (oiter) oiter[b] = info_iter;
        p.rho_upd[b] = rho_updates;
        p.obj[b] = obj;
        p.pri[b] = R.pri;
        p.dua[b] = R.dua;
        p.rho_est[b] = rho_est;
        p.scal[b * 4 + 2] = rho;
    }
}
template <int TT, bool ONE = false, bool EDL = false>
__device__ __noinline__ void finalize_nl(const KParams* gp, long b, double* __restrict__ xo,
                                         double* __restrict__ yo, double cinv, double rho, int status,
                                         int info_iter, int rho_updates, int* ostat, int* oiter) {
    finalize_ph<TT, ONE, EDL>(gp, b, xo, yo, cinv, rho, status, info_iter, rho_updates, ostat, oiter);
}

template <int TT>
__device__ __noinline__ bool factorize_pol_nl(const KParams* gp, long b) {
    KPc& p = kconst(gp);
    SL2 c = carve(p);
    return factorize<TT, KPc, true>(p, c.L, 1.0 / p.delta, p.F + b * (long)p.nb * SS, p.H + b * (long)p.nb * SS,
                                    p.Si + b * (long)p.nb * SS);
}
// sdst: where the S_k^{-1} tiles go (default: the workspace; the two-wave kernel keeps
// them in LDS)
template <int TT, bool ROT = false>
__device__ __forceinline__ bool factorize_ph(const KParams* gp, long b, double rho, double* sdst) {
    KPc& p = kconst(gp);
    SL2 c = carve(p);
    return factorize<TT, KPc, false, ROT>(p, c.L, rho, p.F + b * (long)p.nb * SS, p.H + b * (long)p.nb * SS,
                     sdst ? sdst : p.Si + b * (long)p.nb * SS);
}
// ROT: the Gauss-Jordan steps read and write the tile rows in rotated order (ld_row16)
template <int TT, bool ROT = false>
__device__ __noinline__ bool factorize_nl(const KParams* gp, long b, double rho, double* sdst = nullptr) {
    return factorize_ph<TT, ROT>(gp, b, rho, sdst);
}
// The four-wave kernels' S_k^{-1} tiles in LDS (lds_w2_bytes: after the carve), formed from the
// carve itself: a pointer the compiler sees derived from the LDS array keeps ds_ instructions,
// where one passed in as an argument may become flat accesses -- which wait on the vector-memory
// counter too, i.e. for the factorisation's own workspace stores
template <class KP>
__device__ __forceinline__ double* w4_tiles(const KP& p, const SL2& c) {
    return c.L.Acsc + 2 * ((lds_base_bytes(p) + 15) / 16);
}
// factorize_nl into the LDS tiles (w4_tiles)
template <int TT, bool ROT = false>
__device__ __noinline__ bool factorize_lds_nl(const KParams* gp, long b, double rho) {
    KPc& p = kconst(gp);
    SL2 c = carve(p);
    return factorize<TT, KPc, false, ROT>(p, c.L, rho, p.F + b * (long)p.nb * SS, p.H + b * (long)p.nb * SS,
                                          w4_tiles(p, c));
}
// the one-shot form 3: the G blocks straight into the solve's gl copy (factorize_w4_gl)
template <int TT, bool ROT = false>
__device__ __noinline__ bool factorize_gl_nl(const KParams* gp, long b, double rho) {
    static_assert(TT == 256, "the four-wave kernel");
    KPc& p = kconst(gp);
    SL2 c = carve(p);
    return factorize_w4_gl<ROT>(p, c.L, rho, w4_tiles(p, c), p.F + b * (long)p.nb * SS);
}
// the same with the G blocks to the LDS region after the tiles (the one-shot fused kernel's GL
// form, one_shot_form 2: no workspace round trip) instead of the instance's H tiles
template <int TT, bool ROT = false>
__device__ __noinline__ bool factorize_g_nl(const KParams* gp, long b, double rho) {
    KPc& p = kconst(gp);
    SL2 c = carve(p);
    double* const sg = w4_tiles(p, c);
    return factorize<TT, KPc, false, ROT>(p, c.L, rho, p.F + b * (long)p.nb * SS, sg + (long)p.nb * SS, sg);
}


size_t lds_solve_bytes(const KParams& p);

}  // namespace mpcqp
