// device_common.h -- constants and wave/block primitives shared by the HIP kernels.
#pragma once
#include <hip/hip_runtime.h>

#include "kernels.h"

#ifdef MPCQP_SKEW
// Barrier-race debug build (make skew -> libmpcqp_skew.so; tests/test_skew.py): after every
// workgroup barrier about half of the waves, picked by their wave index and the scalar clock
// (so a different half at each barrier), sleep ~1,300 cycles before going on.  A hand-off
// between waves that lacks a barrier -- a wave reading what another writes, or overwriting
// what another still reads -- then sees the other wave's stale or new data within a few
// barriers, instead of in 1 of ~4 runs (the round-2 y-park race).  Results of a race-free
// kernel are bit-identical to the production build's.
__device__ inline __attribute__((convergent)) void mpcqp_skew_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const unsigned w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const unsigned t = (unsigned)(__builtin_amdgcn_s_memtime() >> 3);
    if (((t ^ (w * 0x9E3779B9u)) >> 7) & 1u) __builtin_amdgcn_s_sleep(20);
}
#define __syncthreads() mpcqp_skew_barrier()
#endif

namespace mpcqp {

// OSQP 0.6 constants (constants.h of the published solver)
#define OSQP_INFTY 1e30
#define MIN_SCALING 1e-4
#define MAX_SCALING 1e4
#define RHO_MIN 1e-6
#define RHO_MAX 1e6
#define RHO_TOL 1e-4
#define RHO_EQ_OVER_RHO_INEQ 1e3
#define DIVISION_TOL (1.0 / OSQP_INFTY)

constexpr int T = kThreads;

// KParams seen through the constant address space.  Out-of-line device functions
// get the device copy KParams::self (a kernel's by-value argument block would be
// copied to scratch for them); re-qualifying that uniform address makes its field
// reads scalar loads instead of per-lane flat loads into VGPRs.
typedef __attribute__((address_space(4))) const KParams KPc;
__device__ __forceinline__ KPc& kconst(const KParams* gp) {
    const unsigned long long a = (unsigned long long)gp;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
    return *(KPc*)(((unsigned long long)hi << 32) | lo);
}
constexpr int S = kS;
constexpr int SS = kS * kS;

// the instance a solve-kernel workgroup works on (KParams::order); kept in an SGPR
__device__ __forceinline__ long instance_of(const KParams& p) {
    return p.order ? (long)__builtin_amdgcn_readfirstlane(p.order[blockIdx.x]) : (long)blockIdx.x;
}

__device__ __forceinline__ double cmax(double a, double b) { return a > b ? a : b; }
__device__ __forceinline__ double cmin(double a, double b) { return a < b ? a : b; }
__device__ __forceinline__ double limit_scaling(double d) {
    d = d < MIN_SCALING ? 1.0 : d;
    return d > MAX_SCALING ? MAX_SCALING : d;
}

// DPP lane permutation of a double: two v_mov_b32_dpp, bound_ctrl set so no copy
// of the old value is needed.  CTRL: 0xB1 quad_perm[1,0,3,2], 0x4E quad_perm[2,3,0,1],
// 0x141 row_half_mirror, 0x140 row_mirror (every lane has a valid source).
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
    int lo = __double2loint(v), hi = __double2hiint(v);
    lo = __builtin_amdgcn_mov_dpp(lo, CTRL, 0xF, 0xF, true);
    hi = __builtin_amdgcn_mov_dpp(hi, CTRL, 0xF, 0xF, true);
    return __hiloint2double(hi, lo);
}

// sum over the 8 lanes of an aligned half-row (lanes 8r..8r+7), result in all 8
__device__ __forceinline__ double reduce8(double v) {
    v += dpp<0xB1>(v);
    v += dpp<0x4E>(v);
    v += dpp<0x141>(v);
    return v;
}

// sum over the 16 lanes of a DPP row, result in all 16
__device__ __forceinline__ double reduce16(double v) {
    v += dpp<0xB1>(v);
    v += dpp<0x4E>(v);
    v += dpp<0x141>(v);
    v += dpp<0x140>(v);
    return v;
}

// DPP with a row mask: rows outside `RM` get an unspecified value (callers only
// read lanes of the written rows)
template <int CTRL, int RM>
__device__ __forceinline__ double dpp_rows(double v) {
    int lo = __double2loint(v), hi = __double2hiint(v);
    lo = __builtin_amdgcn_mov_dpp(lo, CTRL, RM, 0xF, true);
    hi = __builtin_amdgcn_mov_dpp(hi, CTRL, RM, 0xF, true);
    return __hiloint2double(hi, lo);
}

// sum over an aligned 32-lane half-wave; valid in its upper 16 lanes
// (row_bcast:15 adds lane 15 of rows 0/2 into rows 1/3)
__device__ __forceinline__ double reduce32_hi(double v) {
    v = reduce16(v);
    v += dpp_rows<0x142, 0xA>(v);
    return v;
}

// Wave-wide reductions by DPP (rows of 16, then row_bcast:15 / row_bcast:31);
// the result is read from lane 63 (only lanes of the written rows are valid after
// the broadcasts) into a scalar register.
__device__ __forceinline__ double lane63(double v) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), 63),
                            __builtin_amdgcn_readlane(__double2loint(v), 63));
}
__device__ __forceinline__ double wave_max(double v) {
    v = cmax(v, dpp<0xB1>(v));
    v = cmax(v, dpp<0x4E>(v));
    v = cmax(v, dpp<0x141>(v));
    v = cmax(v, dpp<0x140>(v));
    v = cmax(v, dpp_rows<0x142, 0xA>(v));
    v = cmax(v, dpp_rows<0x143, 0xC>(v));
    return lane63(v);
}
__device__ __forceinline__ double wave_sum(double v) {
    v = reduce16(v);
    v += dpp_rows<0x142, 0xA>(v);
    v += dpp_rows<0x143, 0xC>(v);
    return lane63(v);
}

// Workgroup-wide max / sum of K values over TT threads (OSQP c_max semantics per
// comparison).  A one-wave workgroup (TT = 64) reduces in registers only; wider
// ones go through red[] (TT/64 * K slots).
template <int TT, int K>
__device__ __forceinline__ void block_max(double (&v)[K], double* red) {
    if constexpr (TT == 64) {
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = wave_max(v[k]);
    } else {
        constexpr int NW = TT / 64;
        const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const double r = wave_max(v[k]);
            if (lane == 0) red[wid * K + k] = r;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < K; ++k) {
            double r = red[k];
#pragma unroll
            for (int w = 1; w < NW; ++w) r = cmax(r, red[w * K + k]);
            v[k] = r;
        }
        __syncthreads();
    }
}

// block-wide max of K values into out[0..K) (LDS), computed by threads k < K;
// visible to every thread after the trailing barrier.  red needs TT/64*K slots.
template <int TT, int K>
__device__ __forceinline__ void block_max_to(const double (&v)[K], double* red, double* out) {
    constexpr int NW = TT / 64;
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63, t = threadIdx.x;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const double r = wave_max(v[k]);
        if (lane == 0) red[wid * K + k] = r;
    }
    __syncthreads();
    if (t < K) {
        double r = red[t];
#pragma unroll
        for (int w = 1; w < NW; ++w) r = cmax(r, red[w * K + t]);
        out[t] = r;
    }
    __syncthreads();
}

template <int TT, int K>
__device__ __forceinline__ void block_sum(double (&v)[K], double* red) {
    if constexpr (TT == 64) {
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = wave_sum(v[k]);
    } else {
        constexpr int NW = TT / 64;
        const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const double r = wave_sum(v[k]);
            if (lane == 0) red[wid * K + k] = r;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < K; ++k) {
            double r = red[k];
            if constexpr (NW == 4) {
                r = (red[k] + red[K + k]) + (red[2 * K + k] + red[3 * K + k]);
            } else {
#pragma unroll
                for (int w = 1; w < NW; ++w) r += red[w * K + k];
            }
            v[k] = r;
        }
        __syncthreads();
    }
}

// ---- transposed multi-value reductions (the termination check's 17 maxima) ----
// max of two non-negative doubles: v_max_f64 (one instruction; a NaN operand is
// skipped, as OSQP's sequential vec_norm_inf skips it)
__device__ __forceinline__ double vmax(double a, double b) { return __builtin_fmax(a, b); }

// One transposed step over the lane pairs of DPP CTRL: lanes with `upper` keep the
// upper half of the K values, the others the lower half, each max'ed with the
// partner's copy (the odd value out pairs with 0, neutral for the non-negative
// maxima).  K values in, (K+1)/2 out; 2 DPP moves + 5 VALU per value kept.
template <int CTRL, int K>
__device__ __forceinline__ void tmax_step(const double (&in)[K], double (&out)[(K + 1) / 2], bool upper) {
    constexpr int H = (K + 1) / 2;
#pragma unroll
    for (int j = 0; j < H; ++j) {
        const double lo = in[j];
        const double hi = j + H < K ? in[j + H] : 0.0;
        out[j] = vmax(upper ? hi : lo, dpp<CTRL>(upper ? lo : hi));
    }
}

// max with the lane 16 (xor-like: odd/even DPP rows) or 32 (half-waves) away:
// v_permlane16/32_swap of both dwords, every lane keeps the larger value
template <bool HALF>
__device__ __forceinline__ double xmax_swap(double v) {
    const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
    const auto l = HALF ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false)
                        : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto h = HALF ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false)
                        : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    return vmax(__hiloint2double((int)h[0], (int)l[0]), __hiloint2double((int)h[1], (int)l[1]));
}

// Workgroup max of K non-negative values per thread plus workgroup sums of KS values,
// results in every thread.  The maxima are reduced transposed: two DPP steps split the
// K values over the lanes of a quad (lane bits 0, 1), the rest of the wave reduces the
// remaining (K+3)/4 values per lane over the lanes of equal quad position (row_ror 4 / 8,
// permlane16 / 32 swaps), and one LDS round combines the waves -- about a sixth of the
// instructions of K separate DPP trees.  The sums keep block_sum's order (wave_sum, then
// wave 0 + wave 1 + ...), so they are bit-identical to it.  red: 4 * NW * K2 + NW * KS
// doubles, 16-byte aligned.
template <int TT, int K, int KS>
__device__ __forceinline__ void block_max_sum_tr(double (&v)[K], double (&sm)[KS], double* red) {
    constexpr int NW = TT / 64, K1 = (K + 1) / 2, K2 = (K1 + 1) / 2;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    double t1[K1], t2[K2];
    tmax_step<0xB1, K>(v, t1, lane & 1);          // quad_perm [1,0,3,2]: lane ^ 1
    tmax_step<0x4E, K1>(t1, t2, (lane >> 1) & 1);  // quad_perm [2,3,0,1]: lane ^ 2
#pragma unroll
    for (int j = 0; j < K2; ++j) {
        double x = t2[j];
        x = vmax(x, dpp<0x124>(x));  // row_ror:4
        x = vmax(x, dpp<0x128>(x));  // row_ror:8
        x = xmax_swap<false>(x);
        x = xmax_swap<true>(x);
        t2[j] = x;
    }
    double s[KS];
#pragma unroll
    for (int k = 0; k < KS; ++k) s[k] = wave_sum(sm[k]);
    // lane q < 4 (quad position q = b0 + 2 b1) holds value j + K2 b1 + K1 b0
    double* rs = red + 4 * NW * K2;
    if (lane < 4) {
        // (the lane index through an empty asm: the write addresses are formed here, not
        // kept from the kernel's start across a solve loop that has no register to spare)
        int lq = lane;
        asm volatile("" : "+v"(lq));
#pragma unroll
        for (int j = 0; j < K2; ++j) red[(lq * K2 + j) * NW + wid] = t2[j];
    }
    if (lane == 0) {
        int wq = wid;
        asm volatile("" : "+v"(wq));  // (as lq above)
#pragma unroll
        for (int k = 0; k < KS; ++k) rs[wq * KS + k] = s[k];
    }
    __syncthreads();
    if constexpr (NW > 4) {
        // eight waves: thread k < K folds value k over the waves first (every thread
        // loading all K x NW partials would hold them all in registers at once)
        double* const fin = rs + NW * KS;
        if ((int)threadIdx.x < K) {
            const int k = threadIdx.x, b0 = k >= K1, r1 = k - K1 * b0, b1 = r1 >= K2, j = r1 - K2 * b1;
            const double* src = red + ((b0 + 2 * b1) * K2 + j) * NW;
            double r = src[0];
#pragma unroll
            for (int w = 1; w < NW; ++w) r = vmax(r, src[w]);
            fin[k] = r;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = fin[k];
    } else {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int b0 = k >= K1, r1 = k - K1 * b0, b1 = r1 >= K2, j = r1 - K2 * b1;
            const double* src = red + ((b0 + 2 * b1) * K2 + j) * NW;
            double r = src[0];
#pragma unroll
            for (int w = 1; w < NW; ++w) r = vmax(r, src[w]);
            v[k] = r;
        }
    }
#pragma unroll
    for (int k = 0; k < KS; ++k) {
        double r = rs[k];
        if constexpr (NW == 4) {  // block_sum's order for four waves
            r = (rs[k] + rs[KS + k]) + (rs[2 * KS + k] + rs[3 * KS + k]);
        } else {
#pragma unroll
            for (int w = 1; w < NW; ++w) r += rs[w * KS + k];
        }
        sm[k] = r;
    }
    __syncthreads();
}

// Dispatch order for the next solve, sorted by the workgroup that finishes LAST (the
// counting sort of kernels.hip::k_order: 256 bins on iter >> shift, descending, stable in
// instance order within a bin), so no separate kernel and no launch gap follow the solve.
// Every workgroup arrives once on p.done after its instance's iteration count is written;
// the last arrival has seen every count (release / acquire fences around the atomic),
// and no workgroup of this launch still reads the order (all have finished).  smem:
// 257 ints of LDS the caller no longer uses.
template <int TT>
__device__ __forceinline__ void order_epilogue(const KParams& p, int* smem) {
    const long B = gridDim.x;
    if (!p.done || !p.order || B <= p.slots || B > kOrderFuseMax) return;
    const int tid = threadIdx.x;
    int* cnt = smem;
    int* last = smem + 256;
    __syncthreads();  // the instance's results (iter by thread 0) are written
    if (tid == 0) {
        __threadfence();
        *last = atomicAdd(p.done, 1) == (int)(B - 1);
        __threadfence();
    }
    __syncthreads();
    if (!*last) return;
    int shift = 0;
    while ((p.max_iter >> shift) >= 256) ++shift;
    const int* iter = p.iter;
    int* order = const_cast<int*>(p.order);
    auto bin = [&](long i) {
        const int k = __builtin_nontemporal_load(iter + i) >> shift;
        return 255 - (k < 255 ? k : 255);
    };
    for (int k = tid; k < 256; k += TT) cnt[k] = 0;
    __syncthreads();
    for (long i = tid; i < B; i += TT) atomicAdd(&cnt[bin(i)], 1);
    __syncthreads();
    if (tid == 0) {
        int s = 0;
        for (int k = 0; k < 256; ++k) {
            const int c = cnt[k];
            cnt[k] = s;
            s += c;
        }
        *p.done = 0;  // the next launch counts from zero
    }
    __syncthreads();
    for (long i = tid; i < B; i += TT) order[atomicAdd(&cnt[bin(i)], 1)] = (int)i;
}

template <int TT>
__device__ __forceinline__ bool block_any(bool f, int* flag) {
    if constexpr (TT == 64) {
        return __builtin_amdgcn_ballot_w64(f) != 0;
    } else {
        if (threadIdx.x == 0) *flag = 0;
        __syncthreads();
        if (f) *flag = 1;
        __syncthreads();
        bool r = *flag != 0;
        __syncthreads();
        return r;
    }
}

}  // namespace mpcqp
