// Micro-benchmark: the gap between back-to-back kernels on one stream, as a function of
// what the first kernel leaves dirty in L2.  1024 workgroups of 256 threads with 72 KB of
// dynamic LDS (the cfg-2 four-wave kernel's launch shape), each kernel spinning ~400 us so
// the host is always ahead; per workgroup it writes `kb` KB with plain or nontemporal
// stores.  Run under rocprofv3 --kernel-trace to read the gaps; prints hipEvent time per
// launch as well.  hipcc --offload-arch=gfx950 -O3 launch_gap.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <bool NT>
__global__ __launch_bounds__(256) void k(double* out, int per_wg, long long spin) {
    extern __shared__ double lds[];
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < spin) __builtin_amdgcn_s_sleep(8);
    double* o = out + (long)blockIdx.x * per_wg;
    for (int i = threadIdx.x; i < per_wg; i += 256) {
        if (NT) __builtin_nontemporal_store((double)i, o + i);
        else o[i] = (double)i;
    }
    if (threadIdx.x == 0) lds[0] = 1.0;
}

int main(int argc, char** argv) {
    const int nwg = 1024, reps = 12;
    const size_t lds = 72 * 1024;
    // wall_clock64 runs at 100 MHz on gfx9: 40000 ticks = 400 us
    const long long spin = 40000;
    double* d;
    hipMalloc(&d, (size_t)nwg * 8192 * sizeof(double));
    hipFuncSetAttribute((const void*)k<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipFuncSetAttribute((const void*)k<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int kbs[] = {0, 8, 48};
    for (int nt = 0; nt < 2; ++nt)
        for (int kb : kbs) {
            const int per_wg = kb * 1024 / 8;
            hipEventRecord(a, 0);
            for (int r = 0; r < reps; ++r) {
                if (nt) hipLaunchKernelGGL(k<true>, dim3(nwg), dim3(256), lds, 0, d, per_wg, spin);
                else hipLaunchKernelGGL(k<false>, dim3(nwg), dim3(256), lds, 0, d, per_wg, spin);
            }
            hipEventRecord(b, 0);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            printf("%s stores, %2d KB per workgroup (%5.1f MB per launch): %.1f us per launch\n",
                   nt ? "nontemporal" : "plain", kb, nwg * kb / 1024.0, 1000.0 * ms / reps);
        }
    hipFree(d);
    return 0;
}
