// Micro-benchmark: cycles per "LDS write -> s_barrier -> LDS read" step for a
// workgroup of W waves (the dependent chain of the block sweeps).  Prints the
// median over workgroups.  hipcc --offload-arch=gfx950 -O3 barrier_cost.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

template <int MODE>
__global__ void k(long long* out, int iters) {
    __shared__ double buf[1024];
    const int t = threadIdx.x;
    double v = t;
    buf[t] = v;
    __syncthreads();
    const long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
        if (MODE == 0) {  // barrier only
            __syncthreads();
        } else if (MODE == 1) {  // write, barrier, read a neighbour's value
            buf[t] = v;
            __syncthreads();
            v = buf[(t + 1) & (blockDim.x - 1)] * 0.5 + 1.0;
        } else {  // + an 8-lane DPP reduction of a 4-term dot (the sweep's step)
            buf[t] = v;
            __syncthreads();
            const double a = buf[(t & ~7) + 0] * v + buf[(t & ~7) + 1];
            double s = a;
            s += __shfl_xor(s, 1);
            s += __shfl_xor(s, 2);
            s += __shfl_xor(s, 4);
            v = s * 1e-3;
        }
    }
    const long long t1 = clock64();
    if (t == 0) out[blockIdx.x] = (t1 - t0) / iters;
    if (v == 12345.678) out[0] = 0;
}

int main() {
    const int nwg = 256, iters = 2000;
    long long* d;
    hipMalloc(&d, nwg * sizeof(long long));
    std::vector<long long> h(nwg);
    for (int mode = 0; mode < 3; ++mode)
        for (int th : {64, 128, 256, 512, 1024}) {
            if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(nwg), dim3(th), 0, 0, d, iters);
            if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(nwg), dim3(th), 0, 0, d, iters);
            if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(nwg), dim3(th), 0, 0, d, iters);
            hipDeviceSynchronize();
            hipMemcpy(h.data(), d, nwg * sizeof(long long), hipMemcpyDeviceToHost);
            std::sort(h.begin(), h.end());
            printf("mode %d threads %4d: %lld cycles/step (median over %d WGs)\n", mode, th, h[nwg / 2], nwg);
        }
    return 0;
}
