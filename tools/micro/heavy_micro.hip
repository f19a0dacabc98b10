// Heavy-instance micro-benchmark (diagnostic): one 512-thread workgroup per CU, the ADMM
// iteration of a cfg-2-shaped QP (npad 128 in 4 blocks of <= 28 real columns, m 188, gather
// lists of 6) with x~ = M^{-1} b as ONE dense product held in registers (lane = (row pair,
// 14-column segment): 52 row pairs x 8 segments = 416 lanes), and the sweep-operator inversion
// of a 104 x 104 SPD matrix in the same layout.  Prints cycles per iteration / per inversion
// and the inverse's residual ||M K - I||.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int TT = 512, NP = 128, MR = 192, K = 6, SEGW = 14, NRP = 52;

__device__ __forceinline__ double dpp_d(double v, int ctrl);
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
    int lo = __double2loint(v), hi = __double2hiint(v);
    lo = __builtin_amdgcn_mov_dpp(lo, CTRL, 0xF, 0xF, true);
    hi = __builtin_amdgcn_mov_dpp(hi, CTRL, 0xF, 0xF, true);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double reduce8(double v) {
    v += dpp<0xB1>(v);
    v += dpp<0x4E>(v);
    v += dpp<0x141>(v);
    return v;
}

// padded column of compact column c (blocks of 26/25/25/28 real columns at 32 k)
__host__ __device__ inline int padc(int c) {
    const int bs[4] = {26, 25, 25, 28};
    int k = 0;
    while (c >= bs[k]) { c -= bs[k]; ++k; }
    return 32 * k + c;
}

// PROD: 0 no product phase, 1 product without the 8-lane sums, 2 full; ph: per-phase cycles (wave 0)
template <int PROD>
__global__ __launch_bounds__(TT, 1) void k_iter(const double* Mg, const int* colg, const int* rowg, int nit,
                                                 long long* cyc, double* out, long long* ph) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double* Av = sm;                 // 512 A values (+ zero slot at 511)
    double* w = Av + 512;            // MR
    double* rb = w + MR;             // NP
    double* xt = rb + NP;            // NP
    double* rbs = xt + NP;           // 8 x 18: b by segment (PROD 3), banks spread
    const int tid = threadIdx.x, lane = tid & 63;
    for (int e = tid; e < 512; e += TT) Av[e] = e == 511 ? 0.0 : 0.001 * (e % 37) - 0.01;
    for (int i = tid; i < MR; i += TT) w[i] = 0.01 * (i % 7);
    for (int i = tid; i < NP; i += TT) { rb[i] = 0.0; xt[i] = 0.0; }
    // the lane's dense rows: row pair rp = tid / 8, segment s = tid % 8 (block s / 2, half s % 2)
    const int rp = tid >> 3, sg = tid & 7, c0 = 32 * (sg >> 1) + SEGW * (sg & 1);
    double Mr[2][SEGW];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int c = 0; c < SEGW; ++c) Mr[r][c] = tid < 8 * NRP ? Mg[((long)(2 * rp + r) * NP) + c0 + c] : 0.0;
    const int r0 = tid < 8 * NRP ? padc(2 * rp) : 0, r1 = tid < 8 * NRP ? padc(2 * rp + 1) : 0;
    unsigned cg[K], rg[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        cg[k] = tid < NP ? (unsigned)colg[k * NP + tid] : (511u | (0u << 16));
        rg[k] = tid < MR ? (unsigned)rowg[k * MR + tid] : (511u | (0u << 16));
    }
    double X = 0.0, Z = 0.0, y = 0.0;
    const double sigma = 1e-6, alpha = 1.6, q = 0.01 * (tid & 7), rv = 0.1, rvi = 10.0, lo = -1.0, up = 1.0;
    __syncthreads();
    long long t0 = clock64(), tp = t0, pa = 0, pb = 0, pc = 0;
    for (int it = 0; it < nit; ++it) {
        // rhs (columns): x update from x~, b = sigma x - q + A' w
        if (tid < NP) {
            double wv[K], av[K];
#pragma unroll
            for (int k = 0; k < K; ++k) { av[k] = Av[cg[k] & 0xFFFF]; wv[k] = w[cg[k] >> 16]; }
            const double xn = alpha * xt[tid] + (1.0 - alpha) * X;
            X = xn;
            double v = sigma * X - q;
#pragma unroll
            for (int k = 0; k < K; ++k) v += av[k] * wv[k];
            rb[tid] = v;
            if (PROD == 3) {
                const int blk = tid >> 5, c = tid & 31, h = c >= SEGW;
                if (c < 2 * SEGW) rbs[18 * (2 * blk + h) + c - SEGW * h] = v;
            }
        }
        __syncthreads();
        { const long long t = clock64(); pa += t - tp; tp = t; }
        // x~ = M b: 2 rows x 14 columns per lane, 8-lane sums
        if (PROD > 0 && tid < 8 * NRP) {
            double bv[SEGW];
#pragma unroll
            for (int c = 0; c < SEGW; c += 2) {
                const double2 t = PROD == 3 ? *(const double2*)(rbs + 18 * sg + c) : *(const double2*)(rb + c0 + c);
                bv[c] = t.x;
                bv[c + 1] = t.y;
            }
            double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
#pragma unroll
            for (int c = 0; c < SEGW; c += 2) {
                a0 += Mr[0][c] * bv[c];
                a1 += Mr[0][c + 1] * bv[c + 1];
                a2 += Mr[1][c] * bv[c];
                a3 += Mr[1][c + 1] * bv[c + 1];
            }
            const double s0 = PROD >= 2 ? reduce8(a0 + a1) : a0 + a1, s1 = PROD >= 2 ? reduce8(a2 + a3) : a2 + a3;
            if (sg == 0) xt[r0] = s0;
            if (sg == 1) xt[r1] = s1;
        }
        __syncthreads();
        { const long long t = clock64(); pb += t - tp; tp = t; }
        // rows: z~ = A x~, relax, project, y, w
        if (tid < MR) {
            double xv[K], av[K];
#pragma unroll
            for (int k = 0; k < K; ++k) { av[k] = Av[rg[k] & 0xFFFF]; xv[k] = xt[rg[k] >> 16]; }
            double zt = av[0] * xv[0];
#pragma unroll
            for (int k = 1; k < K; ++k) zt += av[k] * xv[k];
            const double zr = alpha * zt + (1.0 - alpha) * Z;
            const double zn = fmin(fmax(zr + rvi * y, lo), up);
            y += rv * (zr - zn);
            Z = zn;
            w[tid] = rv * zn - y;
        }
        __syncthreads();
        { const long long t = clock64(); pc += t - tp; tp = t; }
    }
    const long long t1 = clock64();
    if (tid == 0) { cyc[blockIdx.x] = t1 - t0; ph[3 * blockIdx.x] = pa; ph[3 * blockIdx.x + 1] = pb; ph[3 * blockIdx.x + 2] = pc; }
    if (tid < MR) out[blockIdx.x * 1024 + tid] = Z + X;
}

// Sweep-operator inversion of the SPD 104 x 104 matrix Kg (compact, row-major), in the
// product layout; writes -(sweep result) = K^{-1} to Mo (compact, row-major).
__global__ __launch_bounds__(TT, 1) void k_sweep(const double* Kg, double* Mo, long long* cyc, int reps) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double* rowb = sm;  // 2 x 112: the published pivot row (compact segment order)
    const int tid = threadIdx.x, rp = tid >> 3, sg = tid & 7;
    const bool act = tid < 8 * NRP;
    // compact columns of segment sg: [13 sg, 13 sg + 13) -- 104 = 8 x 13
    constexpr int CW = 13;
    const int cb = CW * sg;
    double a[2][CW];
    long long tot = 0;
    for (int rep = 0; rep < reps; ++rep) {
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int c = 0; c < CW; ++c) a[r][c] = act ? Kg[(2 * rp + r) * 104 + cb + c] : 0.0;
        __syncthreads();
        const long long t0 = clock64();
        // publish row 0
        if (rp == 0 && act) {
#pragma unroll
            for (int c = 0; c < CW; ++c) rowb[cb + c] = a[0][c];
        }
        __syncthreads();
#pragma unroll 1
        for (int p = 0; p < 104; ++p) {
            const double* rw = rowb + (p & 1) * 112;
            double pr[CW];
#pragma unroll
            for (int c = 0; c < CW; ++c) pr[c] = rw[cb + c];
            const double d = rw[p];
            const double ai0 = rw[2 * rp], ai1 = rw[2 * rp + 1];  // column p = row p (symmetric)
            double di = __builtin_amdgcn_rcp(d);
            di = __builtin_fma(di, __builtin_fma(-d, di, 1.0), di);
            di = __builtin_fma(di, __builtin_fma(-d, di, 1.0), di);
            const int prp = p >> 1, pr_ = p & 1;
            const bool own0 = rp == prp && pr_ == 0, own1 = rp == prp && pr_ == 1;
            const double f0 = own0 ? 0.0 : ai0 * di, f1 = own1 ? 0.0 : ai1 * di;
#pragma unroll
            for (int c = 0; c < CW; ++c) {
                a[0][c] = __builtin_fma(-f0, pr[c], a[0][c]);
                a[1][c] = __builtin_fma(-f1, pr[c], a[1][c]);
            }
            // the pivot row: a_pj / d, a_pp = -1 / d; the pivot column: a_ip = a_ip / d (= f)
            const int jp = p - cb;  // the pivot column's slot in this segment (uniform per segment)
            if (own0 || own1) {
#pragma unroll
                for (int c = 0; c < CW; ++c) {
                    const double v = (own0 ? a[0][c] : a[1][c]) * di;
                    if (own0) a[0][c] = v; else a[1][c] = v;
                }
            }
            if (jp >= 0 && jp < CW) {
#pragma unroll
                for (int c = 0; c < CW; ++c)
                    if (c == jp) {
                        a[0][c] = own0 ? -di : f0;
                        a[1][c] = own1 ? -di : f1;
                    }
            }
            // publish row p + 1 (its owners' values after this step)
            if (p + 1 < 104 && act && rp == ((p + 1) >> 1)) {
                double* nw = rowb + ((p + 1) & 1) * 112;
#pragma unroll
                for (int c = 0; c < CW; ++c) nw[cb + c] = ((p + 1) & 1) ? a[1][c] : a[0][c];
            }
            __syncthreads();
        }
        tot += clock64() - t0;
    }
    if (act) {
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int c = 0; c < CW; ++c) Mo[(2 * rp + r) * 104 + cb + c] = -a[r][c];
    }
    if (tid == 0) cyc[blockIdx.x] = tot / reps;
}

int main() {
    const int G = 32, NIT = 2000;
    // SPD test matrix: block-tridiagonal-ish band plus diagonal
    std::vector<double> Kc(104 * 104, 0.0);
    srand(7);
    for (int i = 0; i < 104; ++i)
        for (int j = i; j < 104 && j < i + 30; ++j) {
            const double v = (double)rand() / RAND_MAX - 0.5;
            Kc[i * 104 + j] += v;
            Kc[j * 104 + i] += (i == j) ? 0.0 : v;
        }
    for (int i = 0; i < 104; ++i) Kc[i * 104 + i] = 35.0 + i * 0.1;
    std::vector<double> Mp(NP * NP, 0.0);
    for (int i = 0; i < 104; ++i)
        for (int j = 0; j < 104; ++j) Mp[(size_t)i * NP + padc(j)] = 1e-3 * Kc[i * 104 + j];
    std::vector<int> colg(K * NP), rowg(K * MR);
    for (int k = 0; k < K; ++k) {
        for (int c = 0; c < NP; ++c) colg[k * NP + c] = (int)(((c * 7 + k * 13) % 448) | (((c * 3 + k * 5) % MR) << 16));
        for (int r = 0; r < MR; ++r) rowg[k * MR + r] = (int)(((r * 5 + k * 11) % 448) | (padc((r * 3 + k * 7) % 104) << 16));
    }
    double *dM, *dK, *dMo, *dout;
    int *dc, *dr;
    long long* dcyc;
    CK(hipMalloc(&dM, 8 * NP * NP));
    CK(hipMalloc(&dK, 8 * 104 * 104));
    CK(hipMalloc(&dMo, 8 * 104 * 104));
    CK(hipMalloc(&dout, 8 * 1024 * G));
    CK(hipMalloc(&dc, 4 * K * NP));
    CK(hipMalloc(&dr, 4 * K * MR));
    CK(hipMalloc(&dcyc, 8 * G));
    CK(hipMemcpy(dM, Mp.data(), 8 * NP * NP, hipMemcpyHostToDevice));
    CK(hipMemcpy(dK, Kc.data(), 8 * 104 * 104, hipMemcpyHostToDevice));
    CK(hipMemcpy(dc, colg.data(), 4 * K * NP, hipMemcpyHostToDevice));
    CK(hipMemcpy(dr, rowg.data(), 4 * K * MR, hipMemcpyHostToDevice));
    const size_t lds = 100000;
    CK(hipFuncSetAttribute((const void*)k_sweep, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    std::vector<long long> cyc(G);
    long long* dph;
    CK(hipMalloc(&dph, 8 * 3 * G));
    std::vector<long long> ph(3 * G);
    auto run = [&](auto kern, const char* what) -> int {
        CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        for (int rep = 0; rep < 2; ++rep) {
            hipLaunchKernelGGL(kern, dim3(G), dim3(TT), lds, 0, dM, dc, dr, NIT, dcyc, dout, dph);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(cyc.data(), dcyc, 8 * G, hipMemcpyDeviceToHost));
            CK(hipMemcpy(ph.data(), dph, 8 * 3 * G, hipMemcpyDeviceToHost));
            long long mx = 0, mn = cyc[0];
            for (auto c : cyc) { mx = std::max(mx, c); mn = std::min(mn, c); }
            printf("%s: iteration %.0f .. %.0f cycles; wave 0 phases rhs %.0f product %.0f rows %.0f\n", what,
                   (double)mn / NIT, (double)mx / NIT, (double)ph[0] / NIT, (double)ph[1] / NIT, (double)ph[2] / NIT);
        }
        return 0;
    };
    if (run(k_iter<3>, "full, bank-spread b") || run(k_iter<2>, "full") || run(k_iter<1>, "no 8-lane sums") || run(k_iter<0>, "no product")) return 1;
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_sweep, dim3(G), dim3(TT), lds, 0, dK, dMo, dcyc, 4);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(cyc.data(), dcyc, 8 * G, hipMemcpyDeviceToHost));
        std::vector<double> Mo(104 * 104);
        CK(hipMemcpy(Mo.data(), dMo, 8 * 104 * 104, hipMemcpyDeviceToHost));
        double res = 0.0;
        for (int i = 0; i < 104; ++i)
            for (int j = 0; j < 104; ++j) {
                double s = 0.0;
                for (int k = 0; k < 104; ++k) s += Mo[i * 104 + k] * Kc[k * 104 + j];
                res = std::max(res, std::fabs(s - (i == j ? 1.0 : 0.0)));
            }
        printf("sweep inversion: %lld cycles, ||M K - I||_max = %.3e\n", cyc[0], res);
    }
    return 0;
}
