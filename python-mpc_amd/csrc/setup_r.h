// setup_r.h -- osqp_setup's data scaling (scale_data: Ruiz, 10 passes + cost scaling)
// and row classification (set_rho_vec) for one QP instance, with register-resident
// index lists.  Used by kernels.hip::k_setup_r (256 threads) and by the fused
// setup + solve kernel solve_wave.hip::k_setup_solve_w2 (128 threads).
//
// Plans with one padded column per thread (npad <= TT) and at most RS rows per thread:
// every index the ten Ruiz passes chase is loaded once into registers -- the column's
// A and P gather lists (plan.cpp gcol / gpsym: packed LDS positions, padded with a zero
// slot), the rows' A lists (grow), the (row, column) of the thread's A and P values --
// so a norm is one round of independent LDS reads instead of a chain of index -> value
// loads, and the thread's own column / row scalings stay in registers.  A is kept in
// the padded-CSC order of the solve kernels from the start.  Same operations in the
// same order per value as kernels.hip::k_setup (maxima are order-free; the
// cost-scaling sum keeps block_sum's order, so with npad <= 128 a 128-thread and a
// 256-thread workgroup give the same sum): bit-identical output.
//
// K: gather-list length (>= gather_k), KP (>= p_k), AS / PS: A / P values per thread.
// KEEP: a matrix update (kernels.hip::k_unscale_mat, OSQP 0.6 osqp_update_P_A) -- the data
// is scaled afresh but the iterates x, z, y, the row classes and rho are left as they are.
// sm: LDS, lds_setup_r_bytes(nnzP, nnzA, npad, m, TT).
#pragma once
#include <hip/hip_runtime.h>

#include "device_common.h"
#include "solve_phases.h"
#include "wave_util.h"

namespace mpcqp {

__host__ __device__ inline size_t lds_setup_r_bytes(int nnzP, int nnzA, int npad, int m, int tt = 256) {
    return sizeof(double) * ((size_t)nnzP + 1 + nnzA + 1 + npad + m + (tt > 512 ? tt / 64 : 8)) + 16;
}

// ONE (the one-shot fused setup + solve, mpcqp_set_one_shot): the scaled problem is left in LDS
// where the solve kernel's carve keeps it (solve_phases.h::carve: A, P, bounds, row classes,
// q, x = z = 0) instead of in the workspace -- no later call reads it there; D, E, c and the
// status slots are written as always
// EDL (with ONE; one_shot_form 2): E and D too go to the carve (solve_phases.h::edl_E / edl_D)
template <int TT, int K, int KP, int RS, int AS, int PS, bool KEEP = false, bool ONE = false, bool EDL = false>
__device__ __forceinline__ void setup_r_body(const KParams& p, const long b, const double* __restrict__ Px_in,
                                             const double* __restrict__ Ax_in, const double* __restrict__ q_in,
                                             const double* __restrict__ l_in, const double* __restrict__ u_in,
                                             double* sm) {
    const int tid = threadIdx.x;
    const int n = p.n, m = p.m, npad = p.npad, nnzP = p.nnzP, nnzA = p.nnzA;
    double* Pv = sm;               // [nnzP + 1]  user order, Pv[nnzP] = 0
    double* Ac = Pv + nnzP + 1;    // [nnzA + 1]  padded-CSC order, Ac[nnzA] = 0
    double* Dt = Ac + nnzA + 1;    // [npad]
    double* Et = Dt + npad;        // [m]
    constexpr int NRED = TT > 512 ? TT / 64 : 8;  // block_sum / block_max: one slot per wave
    double* red = Et + m;          // [NRED]
    int* flag = (int*)(red + NRED);
    const unsigned pbase = lds_addr(Pv), abase = lds_addr(Ac);
    // registers: the thread's column pc = tid and rows tid + s * TT
    const int pc = tid;
    const bool colv = pc < npad && p.pad_var[pc] >= 0;
    unsigned cg[K], pg[KP], rg[RS][K];
#pragma unroll
    for (int k = 0; k < K; ++k)
        cg[k] = abase + 8u * (colv ? ((unsigned)p.gcol[(long)k * npad + pc] & 0xFFFFu) : (unsigned)nnzA);
#pragma unroll
    for (int s = 0; s < RS; ++s) {
        const int i = tid + s * TT;
#pragma unroll
        for (int k = 0; k < K; ++k)
            rg[s][k] = abase + 8u * (i < m ? ((unsigned)p.grow[(long)k * m + i] & 0xFFFFu) : (unsigned)nnzA);
    }
#pragma unroll
    for (int k = 0; k < KP; ++k)
        pg[k] = pbase + 8u * (colv ? ((unsigned)p.gpsym[(long)k * npad + pc] & 0xFFFFu) : (unsigned)nnzP);
    const long bm = p.mat_shared ? 0 : b;  // LTI batches: one P, A for every instance
    int ar[AS], ac[AS], pr[PS], pcol[PS];
#pragma unroll
    for (int s = 0; s < AS; ++s) {
        const int e = tid + s * TT;
        const bool in = e < nnzA;
        const int v = in ? p.acsc_v[e] : 0;
        ar[s] = in ? p.acsc_row[e] : 0;
        ac[s] = in ? p.a_c[v] : 0;
        if (in) Ac[e] = Ax_in[bm * nnzA + v];
    }
#pragma unroll
    for (int s = 0; s < PS; ++s) {
        const int v = tid + s * TT;
        const bool in = v < nnzP;
        pr[s] = in ? p.p_r[v] : 0;
        pcol[s] = in ? p.p_c[v] : 0;
        if (in) Pv[v] = Px_in[bm * nnzP + v];
    }
    if (tid == 0) { Pv[nnzP] = 0.0; Ac[nnzA] = 0.0; }
    double qv = colv ? q_in[b * n + p.pad_var[pc]] : 0.0, Dv = 1.0, Ev[RS];
#pragma unroll
    for (int s = 0; s < RS; ++s) Ev[s] = 1.0;
    double c = 1.0;
    __syncthreads();

    for (int it = 0; it < p.scaling; ++it) {
        // compute_inf_norm_cols_KKT / rows + limit_scaling + sqrt + reciprocal
        if (pc < npad) {
            double d = 1.0;
            if (colv) {
                double d1 = 0.0, d2 = 0.0;
#pragma unroll
                for (int k = 0; k < KP; ++k) d1 = vmax(fabs(lds_at(pg[k])), d1);
#pragma unroll
                for (int k = 0; k < K; ++k) d2 = vmax(fabs(lds_at(cg[k])), d2);
                d = 1.0 / sqrt(limit_scaling(vmax(d1, d2)));
            }
            Dt[pc] = d;
        }
#pragma unroll
        for (int s = 0; s < RS; ++s) {
            const int i = tid + s * TT;
            if (i < m) {
                double e = 0.0;
#pragma unroll
                for (int k = 0; k < K; ++k) e = vmax(fabs(lds_at(rg[s][k])), e);
                Et[i] = 1.0 / sqrt(limit_scaling(e));
            }
        }
        __syncthreads();
        // P <- D P D ; A <- E A D ; q <- D q ; D <- D Dt ; E <- E Et
#pragma unroll
        for (int s = 0; s < PS; ++s) {
            const int v = tid + s * TT;
            if (v < nnzP) {
                const double x = Pv[v] * Dt[pr[s]];
                Pv[v] = x * Dt[pcol[s]];
            }
        }
#pragma unroll
        for (int s = 0; s < AS; ++s) {
            const int e = tid + s * TT;
            if (e < nnzA) {
                const double x = Ac[e] * Et[ar[s]];
                Ac[e] = x * Dt[ac[s]];
            }
        }
        if (pc < npad) {
            const double dt = Dt[pc];
            qv *= dt;
            Dv *= dt;
        }
#pragma unroll
        for (int s = 0; s < RS; ++s)
            if (tid + s * TT < m) Ev[s] *= Et[tid + s * TT];
        __syncthreads();
        // cost normalisation: mean column inf-norm of P vs ||q||_inf
        double acc[1] = {0.0}, mq[1] = {0.0};
        if (colv) {
            double d1 = 0.0;
#pragma unroll
            for (int k = 0; k < KP; ++k) d1 = vmax(fabs(lds_at(pg[k])), d1);
            acc[0] = d1;
            mq[0] = fabs(qv);
        }
        block_sum<TT>(acc, red);
        block_max<TT>(mq, red);
        double ct = acc[0] / (double)n;
        double nq = limit_scaling(mq[0]);
        ct = limit_scaling(cmax(ct, nq));
        ct = 1.0 / ct;
#pragma unroll
        for (int s = 0; s < PS; ++s)
            if (tid + s * TT < nnzP) Pv[tid + s * TT] *= ct;
        qv *= ct;
        c *= ct;
        __syncthreads();
    }

    // bounds: clip to +-OSQP_INFTY (python wrapper), validate, scale, classify
    bool bad = false;
    const double rho = cmin(cmax(p.rho0, RHO_MIN), RHO_MAX);
    double lo1[RS], up1[RS];   // (ONE: staged for the solve's LDS carve)
    signed char ct1[RS];
#pragma unroll
    for (int s = 0; s < RS; ++s) {
        const int i = tid + s * TT;
        lo1[s] = up1[s] = 0.0;
        ct1[s] = 0;
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
            if constexpr (ONE) {
                lo1[s] = li;
                up1[s] = ui;
                ct1[s] = t;
            } else {
                p.l[b * m + i] = li;
                p.u[b * m + i] = ui;
            }
            if (!EDL) p.E[b * m + i] = Ev[s];
            if (!KEEP && !ONE) {
                p.ct[b * m + i] = t;
                p.z[b * m + i] = 0.0;
                p.y[b * m + i] = 0.0;
            }
        }
    }
    bad = block_any<TT>(bad, flag);
    if constexpr (ONE) {
        // the scaled data into the solve's carve: every value is read into registers first
        // (the two layouts overlap), then written after a barrier
        static_assert(!KEEP, "a matrix update keeps the workspace");
        double av1[AS], pv1[PS];
#pragma unroll
        for (int s = 0; s < AS; ++s) av1[s] = tid + s * TT < nnzA ? Ac[tid + s * TT] : 0.0;
#pragma unroll
        for (int s = 0; s < PS; ++s) pv1[s] = tid + s * TT < nnzP ? Pv[tid + s * TT] : 0.0;
        __syncthreads();
        SL2 C = carve(p);
#pragma unroll
        for (int s = 0; s < AS; ++s)
            if (tid + s * TT < nnzA) C.L.Acsc[tid + s * TT] = av1[s];
#pragma unroll
        for (int s = 0; s < PS; ++s)
            if (tid + s * TT < nnzP) C.L.Pv[tid + s * TT] = pv1[s];
        const int mp = (m + 63) & ~63;  // (solve_mpad: padded rows inert, l = u = 0)
#pragma unroll
        for (int s = 0; s < RS; ++s) {
            const int i = tid + s * TT;
            if (i < mp) {
                C.L.lo[i] = lo1[s];
                C.L.up[i] = up1[s];
                C.L.ct[i] = ct1[s];
                C.Z[i] = 0.0;
            }
        }
        for (int i = tid + RS * TT; i < mp; i += TT) {  // (rows past RS * TT: padding only)
            C.L.lo[i] = 0.0;
            C.L.up[i] = 0.0;
            C.L.ct[i] = 0;
            C.Z[i] = 0.0;
        }
        if (pc < npad) {
            C.L.qv[pc] = qv;
            C.X[pc] = 0.0;
        }
        if constexpr (EDL) {
            double* const ed = edl_E(p, C);
#pragma unroll
            for (int s = 0; s < RS; ++s)
                if (tid + s * TT < m) ed[tid + s * TT] = Ev[s];
            if (pc < npad) edl_D(p, C)[pc] = Dv;
        }
    } else {
        for (int v = tid; v < nnzP; v += TT) p.Px[b * nnzP + v] = Pv[v];
        for (int e = tid; e < nnzA; e += TT) p.Ax[b * nnzA + e] = Ac[e];
    }
    if (pc < npad) {
        if (!ONE) p.q[b * npad + pc] = qv;
        if (!EDL) p.D[b * npad + pc] = Dv;
        if (!KEEP && !ONE) p.x[b * npad + pc] = 0.0;
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

}  // namespace mpcqp
