// Micro-benchmark: cycles per step of the long-horizon kernel's twisted sweep
// (solve_big.hip::twisted_solve, forward step), taken apart.  One 512-thread workgroup per CU
// (k_solve_b's residency), thread t: half h = t / 256, (i, jg) = (t % 256 / 8, t % 8); a step
// reads w (four doubles at jg + 8 c) and an F row (the same columns), forms two 8-lane dot
// products (S^-1 row from registers, F row), and the row's writer lane stores two values;
// then a workgroup barrier.  Modes:
//   0  the full step
//   1  without the DPP sums (each lane's partial stands in for the sum)
//   2  the full step with a wave barrier instead of s_barrier (no cross-wave order)
//   3  the full step without the stores
//   4  LDS write -> s_barrier -> LDS read of another wave's value (the bare hand-off)
//   5  s_barrier only
//   6  the full step, 256 threads (one wave per SIMD)
//   7  the full step, paired sums: the first DPP level (row_half_mirror) splits the lanes so
//      lanes 0-3 sum the S^-1 row and lanes 4-7 the F row, and lanes 0 and 4 store in one
//      instruction
//   8  the full step without the stores, both sums kept live
// Prints the median over workgroups of cycles per step.  hipcc --offload-arch=gfx950 -O3 sweep_step.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>


template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, true);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double reduce8(double v) {  // 8-lane sums: quad_perm x2, row_half_mirror
    v += dpp<0xB1>(v);
    v += dpp<0x4E>(v);
    v += dpp<0x141>(v);
    return v;
}

template <int MODE, int TT>
__global__ __launch_bounds__(TT, 1) void k(long long* out, double* sink, int iters) {
    extern __shared__ double sm[];
    double* rb = sm;             // 17 blocks x 32
    double* F = sm + 17 * 32;    // 16 rows x 42
    const int t = threadIdx.x, half = t / (TT / 2), u = t % (TT / 2);
    const int i = u / 8 % 32, jg = u % 8;
    for (int e = t; e < 17 * 32 + 16 * 42; e += TT) sm[e] = 1e-3 * (e % 97);
    double inv[4] = {1e-2 * i, 2e-2 * jg, 3e-3, 4e-3};
    __syncthreads();
    const long long t0 = clock64();
    double acc = 0.0;
    for (int it = 0; it < iters; ++it) {
        const int s = it % 8 + 1;
        if (MODE == 5) {
            __syncthreads();
            continue;
        }
        if (MODE == 4) {
            if (jg == 0) rb[(s + 1) % 17 * 32 + i] = acc + 1.0;
            __syncthreads();
            acc += rb[(s + 1) % 17 * 32 + ((i + 8) & 31)] * 0.5;
            continue;
        }
        const int ks = half ? 16 - s : s - 1, kd = half ? 15 - s : s;
        const double* w = rb + ks * 32;
        const double* f = F + (i % 10) * 42;
        const double old = jg == 0 ? rb[kd * 32 + i] : 0.0;
        const double v0 = w[jg], v1 = w[jg + 8], v2 = w[jg + 16], v3 = w[jg + 24];
        const double f0 = f[jg], f1 = f[jg + 8], f2 = f[jg + 16], f3 = f[jg + 24];
        double tt = (inv[0] * v0 + inv[1] * v1) + (inv[2] * v2 + inv[3] * v3);
        double c = (f0 * v0 + f1 * v1) + (f2 * v2 + f3 * v3);
        if (MODE == 7) {
            const bool up = jg >= 4;
            double x = up ? c : tt;
            x += dpp<0x141>(up ? tt : c);
            x += dpp<0xB1>(x);
            x += dpp<0x4E>(x);
            const double old7 = jg == 4 ? rb[kd * 32 + i] : 0.0;
            if ((jg & 3) == 0) rb[(up ? kd : 16) * 32 + i] = up ? old7 - 1e-9 * x : x;
            acc += x;
            __syncthreads();
            continue;
        }
        if (MODE != 1) {
            tt = reduce8(tt);
            c = reduce8(c);
        }
        if (MODE == 8) acc += c;
        if (MODE != 3 && MODE != 8 && jg == 0) {
            rb[32 * 16 + i] = tt;  // (the t row: a block no step reads)
            rb[kd * 32 + i] = old - 1e-9 * c;
        }
        acc += tt;
        if (MODE == 2) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        } else {
            __syncthreads();
        }
    }
    const long long t1 = clock64();
    if (t == 0) out[blockIdx.x] = (t1 - t0) / iters;
    if (acc == 12345.678) sink[t] = acc;
}

template <int MODE, int TT>
static void run(const char* name, int nblk, int iters) {
    long long* d;
    double* sink;
    (void)hipMalloc(&d, nblk * sizeof(long long));
    (void)hipMalloc(&sink, 1024 * sizeof(double));
    const size_t lds = 100 * 1024;  // one workgroup per CU
    (void)hipFuncSetAttribute((const void*)k<MODE, TT>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((k<MODE, TT>), dim3(nblk), dim3(TT), lds, 0, d, sink, iters);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL((k<MODE, TT>), dim3(nblk), dim3(TT), lds, 0, d, sink, iters);
    (void)hipDeviceSynchronize();
    std::vector<long long> h(nblk);
    (void)hipMemcpy(h.data(), d, nblk * sizeof(long long), hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    printf("%-52s %6lld cycles/step (median of %d workgroups)\n", name, h[nblk / 2], nblk);
    (void)hipFree(d);
    (void)hipFree(sink);
}

int main() {
    const int nblk = 256, iters = 4000;
    run<0, 512>("0 full step, 512 threads", nblk, iters);
    run<1, 512>("1 without the DPP sums", nblk, iters);
    run<2, 512>("2 wave barrier instead of s_barrier", nblk, iters);
    run<3, 512>("3 without the stores", nblk, iters);
    run<4, 512>("4 write -> s_barrier -> read", nblk, iters);
    run<5, 512>("5 s_barrier only", nblk, iters);
    run<6 == 6 ? 0 : 0, 256>("6 full step, 256 threads", nblk, iters);
    run<7, 512>("7 paired sums, one store instruction", nblk, iters);
    run<8, 512>("8 without the stores, sums live", nblk, iters);
    return 0;
}
