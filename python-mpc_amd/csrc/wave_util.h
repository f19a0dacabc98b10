// wave_util.h -- LDS addressing helpers shared by the wave-level solve kernels
// (solve_wave.hip, solve_dense.hip): packed gather lists with absolute LDS byte
// addresses and 16-byte LDS reads.
#pragma once
#include <hip/hip_runtime.h>

namespace mpcqp {

// Gather list with absolute LDS byte addresses: (vector address << 16) | (A value
// address); one v_and / v_lshrrev per operand (the wave kernel's LDS is < 64 KiB).
// Built at run start from the plan's (vector index << 16) | (A position) lists.
template <int K>
struct GatherW {
    static_assert(K <= 16, "gather lists are kGS = 16 deep (plan.h)");
    unsigned e[K];
    __device__ __forceinline__ void load(const int* list, int stride, unsigned abase, unsigned vbase) {
        // the stride passes through an empty asm: the K entry addresses are formed here, at
        // each (re)load, instead of being hoisted out of the solve loop as K loop-invariant
        // 64-bit pointers per lane (which the four-wave kernel then spilled to scratch)
        asm volatile("" : "+s"(stride));
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const unsigned raw = (unsigned)list[(long)k * stride];
            e[k] = (((raw >> 16) * 8u + vbase) << 16) | ((raw & 0xFFFFu) * 8u + abase);
        }
    }
    __device__ __forceinline__ void clear(unsigned zero_addr, unsigned vbase) {
#pragma unroll
        for (int k = 0; k < K; ++k) e[k] = (vbase << 16) | zero_addr;
    }
};
// 16-byte LDS reads (ds_read_b128) of two consecutive doubles at a 16-byte aligned address
__device__ __forceinline__ void ld2(const double* p, double& a, double& b) {
    const double2 v = *(const double2*)p;
    a = v.x;
    b = v.y;
}
typedef __attribute__((address_space(3))) const double lds_cdouble;
typedef __attribute__((address_space(3))) const char lds_cchar;
__device__ __forceinline__ double lds_at(unsigned byte_addr) { return *(lds_cdouble*)(unsigned long)byte_addr; }
struct alignas(16) dpair { double x, y; };
__device__ __forceinline__ void lds_at2(unsigned byte_addr, double& a, double& b) {
    __attribute__((address_space(3))) const dpair* v = (__attribute__((address_space(3))) const dpair*)(unsigned long)byte_addr;
    a = v->x;
    b = v->y;
}
__device__ __forceinline__ unsigned lds_addr(const void* p) {  // LDS byte address of a shared pointer
    return (unsigned)(unsigned long)(lds_cchar*)p;
}
// A scalar zero the compiler cannot see through.  Added to an index at a rarely run site
// (a refactorisation, a termination check) it keeps the per-lane address from being formed
// once at the kernel's start and kept -- or spilled to scratch -- across the solve loop.
__device__ __forceinline__ int opaque_zero() {
    int z = 0;
    asm volatile("" : "+s"(z));
    return z;
}
// The same for a (wave-uniform) base pointer: with the instance offset folded in before the
// asm, the per-lane address is the base (SGPRs) plus the lane's 32-bit index.
template <class T>
__device__ __forceinline__ T* opaque_ptr(T* p) {
    asm volatile("" : "+s"(p));
    return p;
}
// The same, keeping the global address space: through the asm a plain pointer becomes a
// generic one, and a flat access counts on the LDS counter as well -- the next LDS wait then
// waits for the global access too (the termination check's D / E / pad_var loads did)
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T* opaque_gptr(T* p) {
    asm volatile("" : "+s"(p));
    return (__attribute__((address_space(1))) T*)p;
}
// A per-lane int through an empty asm (see opaque_zero).
__device__ __forceinline__ int opaque_v(int x) {
    asm volatile("" : "+v"(x));
    return x;
}
// arr[idx] = v in LDS with arr's address through an empty asm: the element address is
// formed at the store (a run's write-back) instead of being kept across the solve loop.
__device__ __forceinline__ void lds_put(const double* arr, int idx, double v) {
    unsigned a = lds_addr(arr);
    asm volatile("" : "+s"(a));
    *(__attribute__((address_space(3))) double*)(unsigned long)(a + 8u * (unsigned)idx) = v;
}

}  // namespace mpcqp
