// Micro-benchmarks of the building blocks of one ADMM phase on gfx950
// (diagnostic; tools/micro/run.sh).  256-thread workgroups, `iters` repetitions,
// cycles per repetition measured with s_memtime by thread 0.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
    int lo = __double2loint(v), hi = __double2hiint(v);
    lo = __builtin_amdgcn_update_dpp(lo, lo, CTRL, 0xF, 0xF, false);
    hi = __builtin_amdgcn_update_dpp(hi, hi, CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double reduce8(double v) {
    v += dpp<0xB1>(v); v += dpp<0x4E>(v); v += dpp<0x141>(v); return v;
}

// mode 0: barrier only; 1: LDS write -> barrier -> dependent LDS read;
// 2: 1 + reduce8 on the value; 3: 2 + 4 independent LDS reads + 4 FMAs before the reduce;
// 4: reduce8 chain only (no barrier); 5: fp64 division chain
__global__ __launch_bounds__(256) void k(int mode, int iters, long long* out, double* sink) {
    __shared__ double buf[2][512];
    const int t = threadIdx.x;
    double v = t * 1e-3;
    buf[0][t] = v; buf[1][t] = v; buf[0][t + 256] = v; buf[1][t + 256] = v;
    __syncthreads();
    long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
        const int p = it & 1;
        if (mode == 0) {
            __syncthreads();
        } else if (mode == 1) {
            buf[p][t] = v;
            __syncthreads();
            v = buf[p][(t * 7 + 3) & 255] * 0.999 + 1e-3;
        } else if (mode == 2) {
            buf[p][t] = v;
            __syncthreads();
            v = reduce8(buf[p][(t * 7 + 3) & 255]) * 0.1;
        } else if (mode == 3) {
            buf[p][t] = v;
            __syncthreads();
            const double* b = buf[p];
            const int j = t & 7;
            double a = b[j] * 1.01 + b[j + 8] * 0.99;
            double c = b[j + 16] * 1.02 + b[j + 24] * 0.98;
            v = reduce8(a + c) * 0.1;
        } else if (mode == 4) {
            v = reduce8(v) * 0.125;
        } else if (mode == 5) {
            v = 1.0 / (v + 1.5);
        }
    }
    long long t1 = clock64();
    if (t == 0) out[blockIdx.x] = t1 - t0;
    if (v == 12345.678) sink[t] = v;
}

int main(int argc, char** argv) {
    const int iters = 2000;
    long long* d;
    double* sink;
    hipMalloc(&d, sizeof(long long) * 4096);
    hipMalloc(&sink, 4096 * sizeof(double));
    const char* names[] = {"barrier", "ldsW+bar+ldsR", "+reduce8", "+4rd4fma+reduce8", "reduce8 only", "fp64 div chain"};
    for (int blocks : {256, 1024}) {
        for (int mode = 0; mode < 6; ++mode) {
            hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, mode, iters, d, sink);
            hipDeviceSynchronize();
            long long h[1024];
            hipMemcpy(h, d, sizeof(long long) * blocks, hipMemcpyDeviceToHost);
            double s = 0;
            for (int i = 0; i < blocks; ++i) s += h[i];
            printf("blocks %4d (%d/CU)  %-18s %7.1f cycles/rep\n", blocks, blocks / 256, names[mode], s / blocks / iters);
        }
    }
    return 0;
}
