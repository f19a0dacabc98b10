// setup_wide.h -- the batch setup for the long-horizon plans (cfg 5: npad 544, m 916,
// nnz(A) 2666): osqp_setup's scale_data (Ruiz, 10 passes + cost scaling) and set_rho_vec's
// row classes for one instance per workgroup, as setup_r.h::setup_r_body does for the plans
// of up to 256 columns, with the same operations in the same order per value: bit-identical
// output.  Used by kernels.hip::k_setup_wide.
//
// A thread holds CS padded columns (pc = tid + c * TT), RS rows (tid + s * TT), AS values of A
// (padded-CSC order, e = tid + s * TT) and PS values of P, with every address the ten passes
// chase in registers (setup_r.h's register lists, here as 16-bit LDS addresses two to a
// register, built once per plan: plan.cpp::build_wide_lists; the workgroup's LDS stays below
// 64 KiB) and, unlike setup_r_body, its own values
// too: LDS keeps only the copies the gathers read.  The gathers read no further
// than the longest list of the wave (a ballot in the prologue), and the cost scaling's sum and
// maximum take one LDS round among the waves that hold columns.
//
// WARM (mpcqp_setup_warm_device): the warm start of the same call follows in the workgroup, as
// kernels.hip::k_warm computes it from the workspace -- x = D^-1 x0, y = E^-1 y0 c, z = A x over
// each row's entries in CSR order -- from the values still on chip, in place of the zeros
// setup writes (x0 / y0 null: those stay zero, as k_warm leaves them).
//
// TT = 1024, CS = 1: one instance per CU (the register lists need ~90 VGPRs), the latency
// form for a few QPs.  TT = 512, CS = 2: two instances per CU (<= 128 VGPRs), for batches --
// the setup is latency-bound (barriers, dependent LDS and fp64 chains), so a second resident
// instance fills the first one's waits.
#pragma once
#include <hip/hip_runtime.h>

#include "device_common.h"
#include "solve_phases.h"
#include "wave_util.h"

namespace mpcqp {

// LDS of setup_wide_body: P, A (each with a zero slot), Dt, Et, 2 reduction slots per 64
// columns of CS * TT, the flag
__host__ __device__ inline size_t lds_setup_wide_bytes(int nnzP, int nnzA, int npad, int m, int ctt) {
    return sizeof(double) * ((size_t)nnzP + 1 + nnzA + 1 + npad + m + ctt / 32) + 16;
}

// slot k of a packed list: 16-bit LDS byte addresses, two to a register
// (sh = 16 and mk = 0xFFFF come through an empty asm once per pass in the loop: the unpacking
// then cannot move out of the loop -- hoisted, it would take a register per address again --
// while the packed words themselves stay untouched, so no spilled copy is rewritten per pass)
__device__ __forceinline__ unsigned slot(const unsigned* g, int k, unsigned sh = 16, unsigned mk = 0xFFFFu) {
    return k & 1 ? g[k >> 1] >> sh : g[k >> 1] & mk;
}

// The wave's span of a gather list of K slots, padded at its end with `pad` (the zero slot):
// 0 = at most one entry in every lane, 1 = at most (K + 1) / 2, 2 = K.  Uniform (a ballot),
// so gather_max branches on scalars.  The pads leave a maximum as it is (vmax(|0|, d) = d for
// the d >= 0 the chain carries), so a shorter chain gives the same value.
template <int K>
__device__ __forceinline__ int wave_span(const unsigned* g, unsigned pad) {
    int len = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) len += slot(g, k) != pad;
    const bool gt1 = __builtin_amdgcn_ballot_w64(len > 1) != 0;
    const bool gth = __builtin_amdgcn_ballot_w64(len > (K + 1) / 2) != 0;
    return gth ? 2 : gt1 ? 1 : 0;
}
template <int K>
__device__ __forceinline__ double gather_max(const unsigned* g, int span, unsigned sh, unsigned mk) {
    double d = 0.0;
    if (span == 0) {
        d = vmax(fabs(lds_at(slot(g, 0, sh, mk))), d);
    } else if (span == 1) {
#pragma unroll
        for (int k = 0; k < (K + 1) / 2; ++k) d = vmax(fabs(lds_at(slot(g, k, sh, mk))), d);
    } else {
#pragma unroll
        for (int k = 0; k < K; ++k) d = vmax(fabs(lds_at(slot(g, k, sh, mk))), d);
    }
    return d;
}

template <int TT, int CS, int RS, int K, int KP, int AS, int PS, bool KEEP, bool WARM = false>
__device__ __forceinline__ void setup_wide_body(const KParams& p, const long b, const double* __restrict__ Px_in,
                                                const double* __restrict__ Ax_in, const double* __restrict__ q_in,
                                                const double* __restrict__ l_in, const double* __restrict__ u_in,
                                                double* sm, const double* __restrict__ x0 = nullptr,
                                                const double* __restrict__ y0 = nullptr) {
    static_assert(!(WARM && KEEP), "a matrix update keeps its iterates");
    constexpr int NW = TT / 64, NV = CS * NW;  // waves; 64-column groups ("virtual waves")
    constexpr bool AVR = TT > 512;  // the thread's A values in registers (the 512-thread form: LDS)
    const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
    const int n = p.n, m = p.m, npad = p.npad, nnzP = p.nnzP, nnzA = p.nnzA;
    double* Pv = sm;             // [nnzP + 1]  user order, Pv[nnzP] = 0
    double* Ac = Pv + nnzP + 1;  // [nnzA + 1]  padded-CSC order, Ac[nnzA] = 0
    double* Dt = Ac + nnzA + 1;  // [npad]
    double* Et = Dt + npad;      // [m]
    double* red = Et + m;        // [2 NV]  column group sums, then maxima
    int* flag = (int*)(red + 2 * NV);
    const unsigned pbase = lds_addr(Pv), abase = lds_addr(Ac);
    const unsigned apad = abase + 8u * (unsigned)nnzA, ppad = pbase + 8u * (unsigned)nnzP;

    static_assert(K == 8 && KP == 4, "the plan's wide lists (plan.cpp::build_wide_lists) hold 8 + 4 slots");
    constexpr int K2 = (K + 1) / 2, KP2 = (KP + 1) / 2;
    // the plan's packed lists are LDS offsets from the dynamic LDS's start: add its address to
    // both halves (no carry: the setup's LDS stays below 64 KiB)
    const unsigned sb = lds_addr(sm) * 0x10001u, apad2 = apad * 0x10001u, ppad2 = ppad * 0x10001u;
    bool colv[CS];
    unsigned cg[CS][K2], pg[CS][KP2], rg[RS][K2];
    int spc[CS], spp[CS], spr[RS];
    double qv[CS], Dv[CS];
#pragma unroll
    for (int c = 0; c < CS; ++c) {
        const int pc = tid + c * TT;
        const int j = pc < npad ? p.pad_var[pc] : -1;
        colv[c] = j >= 0;  // (the padding columns' lists are all pads)
#pragma unroll
        for (int k = 0; k < K2; ++k) cg[c][k] = pc < npad ? (unsigned)p.wcg[(long)k * npad + pc] + sb : apad2;
#pragma unroll
        for (int k = 0; k < KP2; ++k) pg[c][k] = pc < npad ? (unsigned)p.wpg[(long)k * npad + pc] + sb : ppad2;
        spc[c] = wave_span<K>(cg[c], apad);
        spp[c] = wave_span<KP>(pg[c], ppad);
        qv[c] = colv[c] ? q_in[b * n + j] : 0.0;
        Dv[c] = 1.0;
    }
#pragma unroll
    for (int s = 0; s < RS; ++s) {
        const int i = tid + s * TT;
#pragma unroll
        for (int k = 0; k < K2; ++k) rg[s][k] = i < m ? (unsigned)p.wrg[(long)k * m + i] + sb : apad2;
        spr[s] = wave_span<K>(rg[s], apad);
    }
    const long bm = p.mat_shared ? 0 : b;  // LTI batches: one P, A for every instance
    // a value's two scalings: (Et[row] | Dt[col] << 16) for A, (Dt[row] | Dt[col] << 16) for P;
    // A loads in the user's order (coalesced) into its padded-CSC place (csc_pos), and the
    // thread's own values come back from LDS after the barrier below
    unsigned as2[AS], ps2[PS];
    double av[AS], pv[PS];
#pragma unroll
    for (int s = 0; s < AS; ++s) {
        const int e = tid + s * TT;
        as2[s] = e < nnzA ? (unsigned)p.was[e] + sb : 0u;
        if (e < nnzA) Ac[p.csc_pos[e]] = Ax_in[bm * nnzA + e];
    }
#pragma unroll
    for (int s = 0; s < PS; ++s) {
        const int v = tid + s * TT;
        const bool in = v < nnzP;
        ps2[s] = in ? (unsigned)p.wps[v] + sb : 0u;
        pv[s] = in ? Px_in[bm * nnzP + v] : 0.0;
        if (in) Pv[v] = pv[s];
    }
    if (tid == 0) { Pv[nnzP] = 0.0; Ac[nnzA] = 0.0; }
    double Ev[RS];
#pragma unroll
    for (int s = 0; s < RS; ++s) Ev[s] = 1.0;
    double cs = 1.0;
    // the column groups that hold columns, and the waves that use c_t (columns, P values)
    const int nwc = (npad + 63) >> 6;
    const bool use_ct = wid * 64 < max(npad, nnzP);
    __syncthreads();
#pragma unroll
    for (int s = 0; s < AS; ++s) av[s] = AVR && tid + s * TT < nnzA ? Ac[tid + s * TT] : 0.0;

    for (int it = 0; it < p.scaling; ++it) {
        unsigned sh = 16, mk = 0xFFFFu;  // (opaque per pass: see slot)
        asm volatile("" : "+s"(sh), "+s"(mk));
        // compute_inf_norm_cols_KKT / rows + limit_scaling + sqrt + reciprocal
#pragma unroll
        for (int c = 0; c < CS; ++c) {
            const int pc = tid + c * TT;
            if (pc < npad) {
                double d = 1.0;
                if (colv[c]) {
                    const double d1 = gather_max<KP>(pg[c], spp[c], sh, mk);
                    const double d2 = gather_max<K>(cg[c], spc[c], sh, mk);
                    d = 1.0 / sqrt(limit_scaling(vmax(d1, d2)));
                }
                Dt[pc] = d;
            }
        }
#pragma unroll
        for (int s = 0; s < RS; ++s) {
            const int i = tid + s * TT;
            if (i < m) {
                Et[i] = 1.0 / sqrt(limit_scaling(gather_max<K>(rg[s], spr[s], sh, mk)));
            }
        }
        __syncthreads();
        // P <- D P D ; A <- E A D ; q <- D q ; D <- D Dt ; E <- E Et
#pragma unroll
        for (int s = 0; s < PS; ++s) {
            const int v = tid + s * TT;
            if (v < nnzP) {
                const double x = pv[s] * lds_at(ps2[s] & mk);
                pv[s] = x * lds_at(ps2[s] >> sh);
                Pv[v] = pv[s];
            }
        }
#pragma unroll
        for (int s = 0; s < AS; ++s) {
            const int e = tid + s * TT;
            if (e < nnzA) {
                const double x = (AVR ? av[s] : Ac[e]) * lds_at(as2[s] & mk);
                const double y = x * lds_at(as2[s] >> sh);
                Ac[e] = y;
                if (AVR) av[s] = y;
            }
        }
#pragma unroll
        for (int c = 0; c < CS; ++c)
            if (tid + c * TT < npad) {
                const double dt = Dt[tid + c * TT];
                qv[c] *= dt;
                Dv[c] *= dt;
            }
#pragma unroll
        for (int s = 0; s < RS; ++s)
            if (tid + s * TT < m) Ev[s] *= Et[tid + s * TT];
        __syncthreads();
        // cost normalisation: mean column inf-norm of P vs ||q||_inf -- block_sum / block_max's
        // values and order over 64-column groups (the groups past the columns add zeros there:
        // +0 leaves the sum as it is, the maximum takes cmax(., 0) per such group)
#pragma unroll
        for (int c = 0; c < CS; ++c) {
            const int vw = c * NW + wid;
            if (vw < nwc) {  // (uniform: full-wave DPP)
                const double d1 = colv[c] ? gather_max<KP>(pg[c], spp[c], sh, mk) : 0.0;
                const double su = wave_sum(d1), mx = wave_max(colv[c] ? fabs(qv[c]) : 0.0);
                if (lane == 0) {
                    red[vw] = su;
                    red[NV + vw] = mx;
                }
            }
        }
        __syncthreads();
        if (use_ct) {
            double su = red[0], mx = red[NV];
#pragma unroll
            for (int w = 1; w < NV; ++w) {
                if (w < nwc) {
                    su += red[w];
                    mx = cmax(mx, red[NV + w]);
                } else {
                    mx = cmax(mx, 0.0);
                }
            }
            double ct = su / (double)n;
            ct = limit_scaling(cmax(ct, limit_scaling(mx)));
            ct = 1.0 / ct;
#pragma unroll
            for (int s = 0; s < PS; ++s)
                if (tid + s * TT < nnzP) {
                    pv[s] *= ct;
                    Pv[tid + s * TT] = pv[s];
                }
#pragma unroll
            for (int c = 0; c < CS; ++c) qv[c] *= ct;
            cs *= ct;
        }
        __syncthreads();
    }

    // (c: right in the waves that use c_t; the warm start's rows read thread 0's, published
    // by block_any's barriers below)
    if (WARM && tid == 0) red[0] = cs;
    // bounds: clip to +-OSQP_INFTY (python wrapper), validate, scale, classify
    bool bad = false;
    const double rho = cmin(cmax(p.rho0, RHO_MIN), RHO_MAX);
#pragma unroll
    for (int s = 0; s < RS; ++s) {
        const int i = tid + s * TT;
        if (i < m) {
            double li = cmax(l_in[b * m + i], -OSQP_INFTY);
            double ui = cmin(u_in[b * m + i], OSQP_INFTY);
            if (li > ui || li != li || ui != ui) bad = true;
            li = Ev[s] * li;
            ui = Ev[s] * ui;
            signed char t;
            if (li < -OSQP_INFTY * MIN_SCALING && ui > OSQP_INFTY * MIN_SCALING) t = -1;
            else if (ui - li < RHO_TOL) t = 1;
            else t = 0;
            p.l[b * m + i] = li;
            p.u[b * m + i] = ui;
            p.E[b * m + i] = Ev[s];
            if (!KEEP) p.ct[b * m + i] = t;
            if (!KEEP && !WARM) {
                p.z[b * m + i] = 0.0;
                p.y[b * m + i] = 0.0;
            }
        }
    }
    bad = block_any<TT>(bad, flag);
#pragma unroll
    for (int s = 0; s < PS; ++s)
        if (tid + s * TT < nnzP) p.Px[b * nnzP + tid + s * TT] = pv[s];
#pragma unroll
    for (int s = 0; s < AS; ++s)
        if (tid + s * TT < nnzA) p.Ax[b * nnzA + tid + s * TT] = AVR ? av[s] : Ac[tid + s * TT];
#pragma unroll
    for (int c = 0; c < CS; ++c) {
        const int pc = tid + c * TT;
        if (pc < npad) {
            p.q[b * npad + pc] = qv[c];
            p.D[b * npad + pc] = Dv[c];
            if (!KEEP && !WARM) p.x[b * npad + pc] = 0.0;
        }
    }
    if constexpr (WARM) {
        // osqp_warm_start: x = D^-1 x0 (into Dt's LDS, free after the passes), y = E^-1 y0 c,
        // z = A x with A the scaled values on chip (Ac), row entries in CSR order (grow)
        double* xs = Dt;
        const double cw = red[0];
#pragma unroll
        for (int c = 0; c < CS; ++c) {
            const int pc = tid + c * TT;
            if (pc < npad) {
                const int j = p.pad_var[pc];
                const double xv = x0 && j >= 0 ? (1.0 / Dv[c]) * x0[b * n + j] : 0.0;
                xs[pc] = xv;
                p.x[b * npad + pc] = xv;
            }
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < RS; ++s) {
            const int i = tid + s * TT;
            if (i < m) {
                double zs = 0.0;
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const unsigned g = (unsigned)p.grow[(long)k * m + i];
                    if ((g & 0xFFFFu) == (unsigned)nnzA) break;  // (the pads: past the row)
                    zs += Ac[g & 0xFFFFu] * xs[g >> 16];
                }
                p.z[b * m + i] = zs;
                p.y[b * m + i] = y0 ? ((1.0 / Ev[s]) * y0[b * m + i]) * cw : 0.0;
            }
        }
    }
    if (tid == 0) {
        p.scal[b * 4 + 0] = cs;
        p.scal[b * 4 + 1] = 1.0 / cs;
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

}  // namespace mpcqp
