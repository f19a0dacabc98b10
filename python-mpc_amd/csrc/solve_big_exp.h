// solve_big_exp.h -- the long-horizon kernel's forms measured and not taken,
// compiled into the experimental builds only (MPCQP_EXPERIMENTAL: libmpcqp_exp.so and the prof /
// skew diagnostic builds; tests/test_gpu_parity.py runs them against the oracle):
//   TwoSided4 / twisted_solve4   -- the twisted sweep on 256 threads (k_solve_b<256>, variant 15)
//   TwoSidedQ / iface_solve      -- the interface form (MPCQP_BIG_FORM=iface)
//   TwoSidedW / wave_twisted_solve -- the two-wave two-sided kernel (k_solve_b<128>, variant 14)
// Included by solve_big.hip after twisted_solve; the production build sees only the forward
// declarations there (k_solve_b's discarded `if constexpr` branches name them).
#pragma once
// ---------------------------------------------------------------------------
__device__ __forceinline__ double reduce4(double v) {  // sum over an aligned quad, result in all 4
    v += dpp<0xB1>(v);
    v += dpp<0x4E>(v);
    return v;
}

// The twisted sweep on 256 threads (k_solve_b<256>, variant 15, experimental build only: measured
// 43.0 against 35.7 ms on cfg 5, DESIGN.md §10 -- the steps are latency-bound, not issue-bound,
// and one wave per SIMD hides none of it): one wave per SIMD, four lanes per tile row.  Thread t: half h = t / 128 (0 top, 1 bottom), (i, q) = (t % 128 / 4, t % 4):
// lane q of row i holds columns [8 q, 8 q + 8) of every tile of its chain, so a forward step is
// four 16-byte reads of w and four of the F / G row, 16 FMAs and two 2-level quad sums per lane
// -- against twisted_solve's 8 lanes of 4 columns, 3-level sums and two waves per SIMD: the
// 512-thread step issues ~78 instructions on each of two waves per SIMD, which is what a step
// costs there (~940 cycles on cfg 5).  The same sums (association aside) in the same steps.
template <int SL>
struct TwoSided4 {
    double Inv[SL][8];
    __device__ __forceinline__ void load(int nb, int pm, int amax, int bmax, const double* __restrict__ Fg,
                                         const double* __restrict__ Hg, const double* __restrict__ Sg,
                                         double* __restrict__ Fc, double* __restrict__ Gc) {
        constexpr int TT = 256;
        const int tid = threadIdx.x, half = __builtin_amdgcn_readfirstlane(tid >> 7), u = tid & 127, i = u >> 2,
                  q = u & 3;
        const int nbot = nb - 1 - pm;
#pragma unroll
        for (int s = 0; s < SL; ++s) {
            const bool have = half == 0 ? s <= pm : s < nbot;
            const int k = half == 0 ? s : nb - 1 - s;
            const double* src = Sg + (long)(have ? k : 0) * SS + i * S + 8 * q;
#pragma unroll
            for (int c = 0; c < 8; c += 2) {
                const double2 t2 = have ? *(const double2*)(src + c) : make_double2(0.0, 0.0);
                Inv[s][c] = t2.x;
                Inv[s][c + 1] = t2.y;
            }
        }
        for (int o = tid; o < pm * amax * S; o += TT) {  // row q = k amax + r of F_{k+1}
            const int qq = o >> 5, j = o & (S - 1), k = qq / amax, r = qq - k * amax;
            Fc[qq * FGS + j] = Fg[(long)(k + 1) * SS + r * S + j];
        }
        for (int o = tid; o < nbot * bmax * S; o += TT) {
            const int qq = o >> 5, j = o & (S - 1), k = qq / bmax, r = qq - k * bmax;
            Gc[qq * FGS + j] = Hg[(long)(pm + k) * SS + r * S + j];
        }
    }
};

__device__ __forceinline__ double dot8(const double (&a)[8], const double (&v)[8]) {
    return ((a[0] * v[0] + a[1] * v[1]) + (a[2] * v[2] + a[3] * v[3])) +
           ((a[4] * v[4] + a[5] * v[5]) + (a[6] * v[6] + a[7] * v[7]));
}

template <int SL>
__device__ __forceinline__ void twisted_solve4(const TwoSided4<SL>& R, const KParams& p, const double* Fc,
                                               const double* Gc, const int* toffL, const int (&so)[SL],
                                               const int (&fo)[SL], double* rb, double* xt, double* corB,
                                               long long* pacc) {
    constexpr bool PRE = SL <= 10;  // (step offsets formed at the run start: step_offsets<SL, 256>)
    extern __shared__ __attribute__((aligned(16))) double sm[];
#ifdef MPCQP_PHASE_PROF
    long long t0s = clock64();
#define SPH(k) if (pacc && threadIdx.x == 0) { const long long t_ = clock64(); pacc[k] += t_ - t0s; t0s = t_; }
#else
#define SPH(k)
#endif
    int opq = 0;
    asm volatile("" : "+s"(opq));  // keep per-block LDS addresses out of the register budget
    const int tid = threadIdx.x, half = __builtin_amdgcn_readfirstlane(tid >> 7), u = tid & 127, i = u >> 2,
              q = u & 3, c8 = 8 * q + opq;
    const int nb = p.nb, pm = p.pmeet, amax = p.amax, bmax = p.bmax, nbot = nb - 1 - pm;
    const int nst = nbot > pm ? nbot : pm;
    const int nmine = half ? nbot : pm, lim = half ? bmax : amax;
    const int apart = __builtin_amdgcn_readfirstlane(PRE ? so[0] : middle_apart(p, toffL));
    const bool writer = q == 0, lowrank = i < lim;
    const int ir = lowrank ? i : 0;  // F / G row this thread sums (row 0 for the rest: reads stay in range)
    auto ld8 = [](const double* a, double (&v)[8]) __attribute__((always_inline)) {
#pragma unroll
        for (int c = 0; c < 8; c += 2) {
            const double2 t2 = *(const double2*)(a + c);
            v[c] = t2.x;
            v[c + 1] = t2.y;
        }
    };
    // forward: top step s: t_{s-1} = S_{s-1}^{-1} w_{s-1}, w_s -= F_s w_{s-1};
    //          bottom step s (k = nb-1-s): t~_{k+1} = T_{k+1}^{-1} w~_{k+1}, w~_k -= G_k w~_{k+1}
#pragma unroll
    for (int s = 1; s < SL; ++s) {
        if (s <= nst) {
            if (s <= nmine) {
                const int ks = half ? nb - s : s - 1, kd = half ? nb - 1 - s : s;
                const int woff = PRE ? 0 : kd * S + (half ? toffL[kd] : 0);
                const bool mid = half && kd == pm && !apart;
                double* dst = PRE ? sm + (so[s] & 0xFFFF) + i : (mid ? corB : rb) + woff + i;
                const double old = (writer && lowrank && !mid) ? *dst : 0.0;
                double v8[8], f8[8];
                ld8(rb + ks * S + c8, v8);
                const double* f = PRE ? sm + (fo[s] & 0xFFFF) + ir * FGS
                                           : (half ? Gc + (kd - pm) * bmax * FGS : Fc + (s - 1) * amax * FGS) + ir * FGS;
                ld8(f + c8, f8);
                const double t = reduce4(dot8(R.Inv[s - 1], v8));
                const double c = reduce4(dot8(f8, v8));
                if (writer) {
                    xt[ks * S + i] = t;
                    if (lowrank) *dst = mid ? c : old - c;
                }
            }
            __syncthreads();
        }
    }
    SPH(12)
    // middle: x_p = M^{-1} w_p with both chains' corrections, by the top half
    if (half == 0) {
        double w8[8], b8[8];
        ld8(rb + pm * S + c8, w8);
        ld8(corB + pm * S + c8, b8);
#pragma unroll
        for (int c = 0; c < 8; ++c) w8[c] -= b8[c];
#pragma unroll
        for (int s = 0; s < SL; ++s) {
            if (s == pm) {
                const double t = reduce4(dot8(R.Inv[s], w8));
                if (writer) xt[pm * S + i] = t;
            }
        }
    }
    __syncthreads();
    SPH(13)
    // backward: top x_k = t_k - H_k x_{k+1}[0, amax) (k = p-1 .. 0);
    //           bottom x_k = t~_k - G_{k-1}' x_{k-1}[toff_{k-1} + (0, bmax)] (k = p+1 .. nb-1);
    // lane q takes the rows r = q + 4 c (< lim) of the sum
#pragma unroll
    for (int s = 1; s < SL; ++s) {
        if (s <= nst) {
            if (s <= nmine) {
                const int k = half ? pm + s : pm - s;
                const double* x1 = PRE ? sm + (so[s] >> 16) : xt + (half ? (k - 1) * S + toffL[k - 1] : (k + 1) * S);
                // H_k[i][r] = F_{k+1}[r][i] (top), G_{k-1}[r][i] (bottom); rows >= lim read as 0
                const double* h = PRE ? sm + (fo[s] >> 16) + i
                                           : (half ? Gc + (k - 1 - pm) * bmax * FGS : Fc + k * amax * FGS) + i;
                const double tk = xt[k * S + i];
                double hv[4], xv[4];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int r = q + 4 * c, rr = r < lim ? r : 0;
                    hv[c] = h[rr * FGS];
                    xv[c] = x1[rr];
                }
                double a0 = 0.0, a1 = 0.0;
#pragma unroll
                for (int c = 0; c < 4; c += 2) {
                    a0 += q + 4 * c < lim ? hv[c] * xv[c] : 0.0;
                    a1 += q + 4 * c + 4 < lim ? hv[c + 1] * xv[c + 1] : 0.0;
                }
                const double cs = reduce4(a0 + a1);
                asm volatile("" ::"v"(tk));  // (t_k's read stays with the step's other reads)
                if (writer) xt[k * S + i] = tk - cs;
            }
            __syncthreads();
        }
    }
    SPH(14)
#undef SPH
}

// The interface form of the two-sided solve (round 5; experimental build, MPCQP_BIG_FORM=iface).
// twisted_solve runs every forward and backward step of both chains on all 512 threads, one
// workgroup barrier a step: 2 max(p, nb-1-p) + 1 barriers, ~820 cycles a forward step on cfg
// 5 (profiles/r4s2_phase_cfg5.txt, s.A).  But a step only carries a few rows forward: F_s
// (amax x 32) changes only rows [0, amax) of w_s (U_s, block s's first BFS level), and the
// product F_s w_{s-1} reads w_{s-1}'s own updated rows U_{s-1} plus rows that no step changes
// (b_{s-1} as the rhs left it).  So the sequential part is an amax-row recurrence:
//     w_s[U] = b_s[U] - F_s[:, R] b_{s-1}[R] - F_s[:, U] w_{s-1}[U]        (top, s = 1..p)
// (the bottom chain likewise on the window rows W_k = [toff_k, toff_k + bmax) with G_k), and
// backward x_k[U] = t_k[U] - F_{k+1}[:, U]' x_{k+1}[U].  Each chain is run by ONE wave -- wave
// 0 the top, wave 1 the bottom -- ordered by its own instruction stream (LDS fence + wave
// barrier, no s_barrier), lane (r, q) = (lane / 4, lane % 4) taking row r and columns
// [8 q, 8 q + 8) (a quad sum); everything that is not on the recurrence runs on all threads
// between four workgroup barriers:
//   F  the two forward chains (full-row products: the static columns' reads issue with the
//      dynamic ones)                                                   -> barrier
//   T  t_k = S_k^{-1} w_k for every block at once (M^{-1} (w_p - corB) for the middle), the
//      factor's tiles in registers in the quad layout (TwoSidedQ)        -> barrier
//   B  the two backward chains on the U / W rows                        -> barrier
//   X  every other row: x_k = t_k - H_k x_{k+1}[U] (top), t_k - G_{k-1}' x_{k-1}[W] (bottom)
//                                                                       -> barrier
// Same factor (factorize2s), same LDS F / G rows, the same sums term for term up to their
// association.
template <int SL>
struct TwoSidedQ {
    static constexpr int NR = (SL + 1) / 2;  // rounds: two blocks per round and half
    double Inv[NR][8];  // round r, this thread's block slot s = 2 r + sub: Inv_s[i][8 q + c]
    // frows: also copy the F / G rows into LDS (after a factorisation, which uses that region as
    // scratch; a termination check leaves it alone, so a run start after one need not)
    __device__ __forceinline__ void load(int nb, int pm, int amax, int bmax, const double* __restrict__ Fg,
                                         const double* __restrict__ Hg, const double* __restrict__ Sg,
                                         double* __restrict__ Fc, double* __restrict__ Gc, bool frows = true) {
        const int tid = threadIdx.x, half = __builtin_amdgcn_readfirstlane(tid >> 8), u = tid & 255;
        const int sub = u >> 7, i = (u & 127) >> 2, q = u & 3;
        const int nbot = nb - 1 - pm;
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const int s = 2 * r + sub;
            const bool have = half == 0 ? s <= pm : s < nbot;
            const int k = half == 0 ? s : nb - 1 - s;
            const double* src = Sg + (long)(have ? k : 0) * SS + i * S + 8 * q;
#pragma unroll
            for (int c = 0; c < 8; c += 2) {
                const double2 t2 = have ? *(const double2*)(src + c) : make_double2(0.0, 0.0);
                Inv[r][c] = t2.x;
                Inv[r][c + 1] = t2.y;
            }
        }
        if (!frows) return;
        for (int o = tid; o < pm * amax * S; o += TB) {  // row q = k amax + r of F_{k+1}
            const int qq = o >> 5, j = o & (S - 1), k = qq / amax, r = qq - k * amax;
            Fc[qq * FGS + j] = Fg[(long)(k + 1) * SS + r * S + j];
        }
        for (int o = tid; o < nbot * bmax * S; o += TB) {
            const int qq = o >> 5, j = o & (S - 1), k = qq / bmax, r = qq - k * bmax;
            Gc[qq * FGS + j] = Hg[(long)(pm + k) * SS + r * S + j];
        }
    }
};

__device__ __forceinline__ void chain_sync() {  // one wave's LDS stores before its later loads
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// toff[k] of the lane's wave-uniform k: the window offsets are held one per lane (lane k, loaded
// once per solve), so a step forms its addresses without an LDS round trip
__device__ __forceinline__ int toff_of(int tv, int k) { return __builtin_amdgcn_readlane(tv, k); }

// The middle block p's top rows [0, amax) and window [toff_p, toff_p + bmax) must be disjoint
// (KParams::ifok): both chains then update w_p in place, and t_p = M^{-1} w_p needs no correction.
template <int SL>
__device__ __forceinline__ void iface_solve(const TwoSidedQ<SL>& R, const KParams& p, const double* __restrict__ Fc,
                                            const double* __restrict__ Gc, const int tv, double* __restrict__ rb,
                                            double* __restrict__ xt, double* __restrict__ tt,
                                            double* __restrict__ xu, long long* pacc, long long* pw) {
    // rb: the rhs, updated in place by the forward chains; tt: t_k = Inv_k w_k (T); xu: the
    // backward chains' U / W rows; xt: x~ (X writes every row).  Four distinct LDS arrays, so
    // each phase's loads issue ahead of its stores.
#ifdef MPCQP_PHASE_PROF
    long long t0s = clock64();
#define SPH(k) if (pacc && threadIdx.x == 0) { const long long t_ = clock64(); pacc[k] += t_ - t0s; t0s = t_; }
    // a wave's own time in a sub-phase (lane 0 keeps it: pw[] in its registers)
    long long tw = clock64();
#define WPH(k) if (pw && (threadIdx.x & 63) == 0) { const long long t_ = clock64(); pw[k] += t_ - tw; tw = t_; }
#define WRS() if (pw) tw = clock64();
#else
#define SPH(k)
#define WPH(k)
#define WRS()
#endif
    const int tid = threadIdx.x, w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int nb = p.nb, pm = p.pmeet, amax = p.amax, bmax = p.bmax, nbot = nb - 1 - pm;
    const int half = w >> 2;
    // the chains: wave 0 the top one, wave 1 the bottom one (waves 0 and 1 sit on different
    // SIMDs -- a workgroup's waves go round the SIMDs 0, 2, 1, 3 -- where waves 0 and 4 share one)
    constexpr int WB = 1;
    const int r = lane >> 2, q = lane & 3;  // chain lanes: row r, columns [8 q, 8 q + 8)
    // ---- F: the forward chains (wave 0 top, wave 1 bottom).  Lanes past the chain's rows take
    // row 0 and store row 0's value again (the same sum): no lane mask in the chain ----
    // Each step's F / G row (static) is loaded one step ahead, after the step's dynamic reads, so
    // the step waits only for the rows the previous step wrote (LDS returns in order); two steps
    // per loop pass with two row buffers (a copy between them made the compiler wait for the
    // prefetch before the step's sum).
    if (w == 0 || w == WB) {
        const bool top = w == 0;
        const int lim = top ? amax : bmax, ir = r < lim ? r : 0, nst = top ? pm : nbot;
        // step s (1-based): the row block and its source / destination
        auto rowp = [&](int s) __attribute__((always_inline)) {
            return A16((top ? Fc + ((s - 1) * amax + ir) * FGS : Gc + ((nb - 1 - s - pm) * bmax + ir) * FGS) + 8 * q);
        };
        auto load = [&](int s, double2 (&f)[4]) __attribute__((always_inline)) {
            const double* fp = rowp(s);
#pragma unroll
            for (int c = 0; c < 4; ++c) f[c] = *(const double2*)(fp + 2 * c);
        };
        auto step = [&](int s, const double2 (&fc)[4], double2 (&fn)[4]) __attribute__((always_inline)) {
            const int src = top ? s - 1 : nb - s, dsb = top ? s : nb - 1 - s;
            const double* v = A16(rb + src * S + 8 * q);
            double* dst = rb + dsb * S + (top ? 0 : toff_of(tv, dsb)) + ir;
            double2 v2[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) v2[c] = *(const double2*)(v + 2 * c);
            const double old = *dst;
            load(s < nst ? s + 1 : s, fn);
            double a0 = 0.0, a1 = 0.0;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                a0 = __builtin_fma(fc[c].x, v2[c].x, a0);
                a1 = __builtin_fma(fc[c].y, v2[c].y, a1);
            }
            *dst = old - reduce4(a0 + a1);
            chain_sync();
        };
        double2 fa[4], fb[4];
        load(1, fa);
#pragma unroll 1
        for (int s = 1; s <= nst; s += 2) {
            step(s, fa, fb);
            if (s + 1 <= nst) step(s + 1, fb, fa);
        }
        WPH(0)
    }
    __syncthreads();
    SPH(12)
    WRS()
    // ---- T: t_k = Inv_k w_k, every block of the half at once (quad layout; a slot past the
    // half's blocks reads block 0 and stores to the spare row of tt) ----
    const int u = tid & 255, sub = __builtin_amdgcn_readfirstlane(u >> 7), i = (u & 127) >> 2, qq = u & 3;
#pragma unroll
    for (int rr = 0; rr < TwoSidedQ<SL>::NR; ++rr) {
        const int s = 2 * rr + sub;
        const bool have = half == 0 ? s <= pm : s < nbot;
        const int k = have ? (half == 0 ? s : nb - 1 - s) : 0;
        const double* v = A16(rb + k * S + 8 * qq);
        double a0 = 0.0, a1 = 0.0;
#pragma unroll
        for (int c = 0; c < 8; c += 2) {
            const double2 v2 = *(const double2*)(v + c);
            a0 = __builtin_fma(R.Inv[rr][c], v2.x, a0);
            a1 = __builtin_fma(R.Inv[rr][c + 1], v2.y, a1);
        }
        const double t = reduce4(a0 + a1);
        if (have) tt[k * S + i] = t;
    }
    if (w == 0) { WPH(4) }
    __syncthreads();
    SPH(13)
    WRS()
    // ---- B: the backward chains on the U (top) / W (bottom) rows, into xu (block p: t_p).  The
    // step's H column (four strided reads) and t value are static: loaded one step ahead, two
    // steps per loop pass with two buffers (as the forward chains) ----
    if (w == 0 || w == WB) {
        const bool top = w == 0;
        const int lim = top ? amax : bmax, ir = r < lim ? r : 0;
        const int j0 = min(4 * q, lim - 1), j1 = min(4 * q + 1, lim - 1), j2 = min(4 * q + 2, lim - 1),
                  j3 = min(4 * q + 3, lim - 1);
        const double m0 = 4 * q < lim ? 1.0 : 0.0, m1 = 4 * q + 1 < lim ? 1.0 : 0.0,
                     m2 = 4 * q + 2 < lim ? 1.0 : 0.0, m3 = 4 * q + 3 < lim ? 1.0 : 0.0;
        // step s = 1 .. nst: block k = p - s (top, x_k[U] from x_{k+1}[U]) or p + s (bottom,
        // x_k[W_k] from x_{k-1}[W_{k-1}])
        const int nst = top ? pm - 1 : nbot - 1;
        struct Ops { double h0, h1, h2, h3, t; };
        auto blk = [&](int s) __attribute__((always_inline)) { return top ? pm - s : pm + s; };
        auto load = [&](int s, Ops& o) __attribute__((always_inline)) {
            const int k = blk(s);
            const int tk = top ? 0 : toff_of(tv, k);
            // H_k[r][j]: F_{k+1}[j][r] (top) / G_{k-1}[j][toff_k + r] (bottom)
            const double* h = top ? Fc + k * amax * FGS + ir : Gc + (k - 1 - pm) * bmax * FGS + tk + ir;
            o.h0 = m0 * h[j0 * FGS];
            o.h1 = m1 * h[j1 * FGS];
            o.h2 = m2 * h[j2 * FGS];
            o.h3 = m3 * h[j3 * FGS];
            o.t = tt[k * S + tk + ir];
        };
        auto step = [&](int s, const Ops& oc, Ops& on) __attribute__((always_inline)) {
            const int k = blk(s), kn = top ? k + 1 : k - 1;
            const double* xv = (kn == pm ? tt : xu) + kn * S + (top ? 0 : toff_of(tv, kn));
            const double x0 = xv[j0], x1 = xv[j1], x2 = xv[j2], x3 = xv[j3];
            load(s < nst ? s + 1 : s, on);
            const double a0 = __builtin_fma(oc.h2, x2, oc.h0 * x0), a1 = __builtin_fma(oc.h3, x3, oc.h1 * x1);
            xu[k * S + (top ? 0 : toff_of(tv, k)) + ir] = oc.t - reduce4(a0 + a1);
            chain_sync();
        };
        if (nst >= 1) {
            Ops oa, ob;
            load(1, oa);
#pragma unroll 1
            for (int s = 1; s <= nst; s += 2) {
                step(s, oa, ob);
                if (s + 1 <= nst) step(s + 1, ob, oa);
            }
        }
        WPH(2)
    }
    __syncthreads();
    SPH(8)
    WRS()
    // ---- X: every row of x~ -- the chains' rows from xu, block p from tt, the rest
    //   top:    x_k = t_k - H_k x_{k+1}[U]       (H_k = F_{k+1}'),   k = 0 .. p-1
    //   bottom: x_k = t_k - G_{k-1}' x_{k-1}[W], k = p+1 .. nb-1;  the middle block p = t_p ----
    {
        const int lim = half ? bmax : amax;
        const int j0 = min(4 * qq, lim - 1), j1 = min(4 * qq + 1, lim - 1), j2 = min(4 * qq + 2, lim - 1),
                  j3 = min(4 * qq + 3, lim - 1);
        const double m0 = 4 * qq < lim ? 1.0 : 0.0, m1 = 4 * qq + 1 < lim ? 1.0 : 0.0,
                     m2 = 4 * qq + 2 < lim ? 1.0 : 0.0, m3 = 4 * qq + 3 < lim ? 1.0 : 0.0;
        // the top half takes blocks 0 .. p (block p: a copy of t_p), the bottom half p+1 .. nb-1
        const int nmine = half ? nbot : pm + 1;
#pragma unroll
        for (int rr = 0; rr < TwoSidedQ<SL>::NR; ++rr) {
            const int s = 2 * rr + sub;
            if (s < nmine) {
                const int k = half == 0 ? s : pm + 1 + s;
                const bool mid = half == 0 && k == pm;
                bool done;         // row i of block k was carried by the backward chain
                const double* hv;  // H_k[i][j] (top) / G_{k-1}[j][i] (bottom), j = 4 qq + c
                const double* xv;  // x_{k+1}[j] (top) / x_{k-1}[toff_{k-1} + j] (bottom)
                if (half == 0) {
                    done = k >= 1 && i < amax;
                    hv = Fc + (mid ? 0 : k * amax) * FGS + i;
                    xv = (k + 1 == pm ? tt : xu) + (mid ? 0 : (k + 1) * S);
                } else {
                    const int tk = toff_of(tv, k);
                    done = k <= nb - 2 && i >= tk && i < tk + bmax;
                    hv = Gc + (k - 1 - pm) * bmax * FGS + i;
                    xv = (k - 1 == pm ? tt : xu) + (k - 1) * S + toff_of(tv, k - 1);
                }
                const double tk = tt[k * S + i], xc = xu[k * S + i];
                const double h0 = m0 * hv[j0 * FGS], h1 = m1 * hv[j1 * FGS], h2 = m2 * hv[j2 * FGS],
                             h3 = m3 * hv[j3 * FGS];
                const double a0 = __builtin_fma(h2, xv[j2], h0 * xv[j0]), a1 = __builtin_fma(h3, xv[j3], h1 * xv[j1]);
                const double acc = reduce4(a0 + a1);
                xt[k * S + i] = mid ? tk : (done ? xc : tk - acc);
            }
        }
    }
    if (w == 0) { WPH(5) }
    __syncthreads();
    SPH(14)
#undef SPH
#undef WPH
#undef WRS
}

// ---------------------------------------------------------------------------
// The two-wave variant (k_solve_b<128, ...>: nb <= 8, cfg 3/4's slack layout): one
// wave per chain, so a sweep step is ordered by the wave's own instruction stream
// (LDS fences + wave_barrier, no s_barrier) and the two chains run side by side;
// only the meeting point needs the workgroup.  Lane (i, h) = (lane / 2, lane % 2)
// holds Inv[s][c] = Inv_s[i][16 h + c] (c < 16) of its chain's slot-s tile; a tile
// row is a 2-lane sum.  F / G rows live in LDS (FGS stride) for the low-rank updates
// (rows < amax / bmax, the same lanes) and, transposed, for the backward sweep.
// rb is updated in place: the destination rows' old values are read off the
// critical path; the bottom chain's correction of the middle block goes to corB
// (negated).
template <int NS>
struct TwoSidedW {
    double Inv[NS][16];
    __device__ __forceinline__ void load(int nb, int pm, int amax, int bmax, const double* __restrict__ Fg,
                                         const double* __restrict__ Hg, const double* __restrict__ Sg,
                                         double* __restrict__ Fc, double* __restrict__ Gc) {
        const int tid = threadIdx.x, wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63,
                  i = lane >> 1, h = lane & 1;
        const int nbot = nb - 1 - pm;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const bool have = wv == 0 ? s <= pm : s < nbot;
            const int k = wv == 0 ? s : nb - 1 - s;
            const double* src = Sg + (long)k * SS + i * S + 16 * h;
#pragma unroll
            for (int c = 0; c < 16; c += 2) {
                double2 t2 = have ? *(const double2*)(src + c) : make_double2(0.0, 0.0);
                Inv[s][c] = t2.x;
                Inv[s][c + 1] = t2.y;
            }
        }
        for (int o = tid; o < pm * amax * S; o += 128) {
            const int q = o >> 5, j = o & (S - 1), k = q / amax, r = q - k * amax;
            Fc[q * FGS + j] = Fg[(long)(k + 1) * SS + r * S + j];
        }
        for (int o = tid; o < nbot * bmax * S; o += 128) {
            const int q = o >> 5, j = o & (S - 1), k = q / bmax, r = q - k * bmax;
            Gc[q * FGS + j] = Hg[(long)(pm + k) * SS + r * S + j];
        }
    }
};

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int NS>
__device__ __forceinline__ void wave_twisted_solve(const TwoSidedW<NS>& R, const KParams& p, const double* Fc,
                                                   const double* Gc, const int* toffL, double* rb, double* xt,
                                                   double* corB, long long* pacc) {
#ifdef MPCQP_PHASE_PROF
    long long t0s = clock64();
#define SPH(k) if (pacc && threadIdx.x == 0) { const long long t_ = clock64(); pacc[k] += t_ - t0s; t0s = t_; }
#else
#define SPH(k)
#endif
    int opq = 0;
    asm volatile("" : "+s"(opq));
    const int tid = threadIdx.x, wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = (tid & 63) + opq,
              i = lane >> 1, h = lane & 1;
    const int nb = p.nb, pm = p.pmeet, amax = p.amax, bmax = p.bmax, nbot = nb - 1 - pm;
    const int nmine = wv ? nbot : pm, lim = wv ? bmax : amax;
    const bool writer = h == 0, lowrank = i < lim;
#pragma unroll
    for (int s = 1; s <= NS; ++s) {
        if (s <= nmine) {
            const int ks = wv ? nb - s : s - 1, kd = wv ? nb - 1 - s : s;
            const bool mid = wv && kd == pm;
            double* dst = mid ? corB + i : rb + kd * S + (wv ? toffL[kd] : 0) + i;
            const double old = (writer && lowrank && !mid) ? *dst : 0.0;
            const double* v = A16(rb + ks * S + 16 * h);
            double vv[16];
#pragma unroll
            for (int c = 0; c < 16; c += 2) {
                const double2 t2 = *(const double2*)(v + c);
                vv[c] = t2.x;
                vv[c + 1] = t2.y;
            }
            double a0 = 0.0, a1 = 0.0;
#pragma unroll
            for (int c = 0; c < 16; c += 2) {
                a0 += R.Inv[s - 1][c] * vv[c];
                a1 += R.Inv[s - 1][c + 1] * vv[c + 1];
            }
            double t = a0 + a1;
            t += dpp<0xB1>(t);
            if (lowrank) {
                const double* f = A16((wv ? Gc + (kd - pm) * bmax * FGS : Fc + (s - 1) * amax * FGS) + i * FGS + 16 * h);
                double b0 = 0.0, b1 = 0.0;
#pragma unroll
                for (int c = 0; c < 16; c += 2) {
                    const double2 f2 = *(const double2*)(f + c);
                    b0 += f2.x * vv[c];
                    b1 += f2.y * vv[c + 1];
                }
                double cc = b0 + b1;
                cc += dpp<0xB1>(cc);
                if (writer) *dst = old - cc;
            }
            if (writer) xt[ks * S + i] = t;
            wave_sync();
        }
    }
    __syncthreads();
    SPH(12)
    if (wv == 0) {  // middle: x_p = M^{-1} (w_p with the bottom chain's correction in corB)
        const int toffp = toffL[pm];
        const double* v = A16(rb + pm * S + 16 * h);
        double vv[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) {
            const int a = 16 * h + c - toffp;
            vv[c] = v[c] + ((pm < nb - 1 && a >= 0 && a < bmax) ? corB[a & 15] : 0.0);
        }
        double t = 0.0;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            if (s == pm) {
                double a0 = 0.0, a1 = 0.0;
#pragma unroll
                for (int c = 0; c < 16; c += 2) {
                    a0 += R.Inv[s][c] * vv[c];
                    a1 += R.Inv[s][c + 1] * vv[c + 1];
                }
                t = a0 + a1;
            }
        }
        t += dpp<0xB1>(t);
        if (writer) xt[pm * S + i] = t;
    }
    __syncthreads();
    SPH(13)
#pragma unroll
    for (int s = 1; s <= NS; ++s) {
        if (s <= nmine) {
            const int k = wv ? pm + s : pm - s;
            const double* x1 = xt + (wv ? (k - 1) * S + toffL[k - 1] : (k + 1) * S);
            const double* hr = (wv ? Gc + (k - 1 - pm) * bmax * FGS : Fc + k * amax * FGS) + i;
            const double tk = xt[k * S + i];
            double a0 = 0.0, a1 = 0.0;
#pragma unroll
            for (int c = 0; c < 8; c += 2) {
                const int r0 = h + 2 * c, r1 = h + 2 * c + 2;
                if (r0 < lim) a0 += hr[r0 * FGS] * x1[r0];
                if (r1 < lim) a1 += hr[r1 * FGS] * x1[r1];
            }
            double a = a0 + a1;
            a += dpp<0xB1>(a);
            if (writer) xt[k * S + i] = tk - a;
            wave_sync();
        }
    }
    __syncthreads();
    SPH(14)
#undef SPH
}

