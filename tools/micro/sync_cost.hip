// Micro-benchmark: cycles per dependent exchange step for a 256-thread (four-wave)
// workgroup, the hand-offs of the four-wave ADMM iteration (solve_wave.hip::solve_w4_body):
//   mode 0: s_barrier only
//   mode 1: ds_write_b64 -> __syncthreads -> ds_read_b64 of another wave's value
//   mode 2: ds_write_b64 -> wave barrier (release/acquire fences) -> ds_read_b64 in the wave
//   mode 3: mode 1 with a 3-read gather + 3 FMAs before the write (the rhs / rows phases)
//   mode 4: mode 2 with the same gather + FMAs
// Two workgroups per CU (the four-wave kernel's residency) unless argv[1] == "1".
// Prints the median over workgroups.  hipcc --offload-arch=gfx950 -O3 sync_cost.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

template <int MODE>
__global__ __launch_bounds__(256, 2) void k(long long* out, int iters) {
    __shared__ double buf[512];
    const int t = threadIdx.x;
    double v = t * 1e-3;
    buf[t] = v;
    buf[256 + t] = v;
    __syncthreads();
    const int other = (t + 64) & 255;          // a lane of the next wave
    const int mine = (t & ~63) | ((t + 1) & 63);  // a lane of the same wave
    const long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
        if (MODE == 0) {
            __syncthreads();
        } else if (MODE == 1 || MODE == 3) {
            double x = v;
            if (MODE == 3) {
                const double a = buf[256 + ((t * 7) & 255)], b = buf[256 + ((t * 13) & 255)],
                             c = buf[256 + ((t * 29) & 255)];
                x = v * a + b;
                x = x * c + v;
                x = x * 0.5 + a;
            }
            buf[t] = x;
            __syncthreads();
            v = buf[other] * 0.5 + 1.0;
        } else {
            double x = v;
            if (MODE == 4) {
                const double a = buf[256 + ((t * 7) & 255)], b = buf[256 + ((t * 13) & 255)],
                             c = buf[256 + ((t * 29) & 255)];
                x = v * a + b;
                x = x * c + v;
                x = x * 0.5 + a;
            }
            buf[t] = x;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            v = buf[mine] * 0.5 + 1.0;
        }
    }
    const long long t1 = clock64();
    if (t == 0) out[blockIdx.x] = (t1 - t0) / iters;
    if (v == 12345.678) out[0] = 0;
}

int main(int argc, char** argv) {
    const int per_cu = (argc > 1 && !strcmp(argv[1], "1")) ? 1 : 2;
    const int nwg = 256 * per_cu, iters = 4000;
    long long* d;
    hipMalloc(&d, nwg * sizeof(long long));
    std::vector<long long> h(nwg);
    const char* names[] = {"s_barrier only", "write->syncthreads->read (other wave)",
                           "write->wave barrier->read (same wave)", "gather3+fma3, write->syncthreads->read",
                           "gather3+fma3, write->wave barrier->read"};
    for (int mode = 0; mode < 5; ++mode) {
        if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(nwg), dim3(256), 0, 0, d, iters);
        if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(nwg), dim3(256), 0, 0, d, iters);
        if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(nwg), dim3(256), 0, 0, d, iters);
        if (mode == 3) hipLaunchKernelGGL(k<3>, dim3(nwg), dim3(256), 0, 0, d, iters);
        if (mode == 4) hipLaunchKernelGGL(k<4>, dim3(nwg), dim3(256), 0, 0, d, iters);
        hipDeviceSynchronize();
        hipMemcpy(h.data(), d, nwg * sizeof(long long), hipMemcpyDeviceToHost);
        std::sort(h.begin(), h.end());
        printf("%d WG/CU  mode %d  %-44s  median %lld  p10 %lld  p90 %lld cycles/step\n", per_cu, mode, names[mode],
               h[nwg / 2], h[nwg / 10], h[nwg * 9 / 10]);
    }
    hipFree(d);
    return 0;
}
