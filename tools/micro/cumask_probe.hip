// CU-mask probe (diagnostic): does hipExtStreamCreateWithCUMask confine a stream's
// workgroups to the masked CUs on this box, which mask bit lands on which (XCC, CU), and can a
// one-workgroup-per-CU "heavy" launch run beside a many-workgroup "bulk" launch on the
// complementary mask?  Also times the cross-stream event hand-off of a two-stream step.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <map>
#include <set>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__device__ inline unsigned cu_id() {
    const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
    const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11));
    return ((xcc & 15u) << 16) | ((hw >> 8) & 0xFFu);  // (xcc, se / sh / cu bits)
}

__global__ void k_hold(unsigned* o, long long* t, int us) {
    extern __shared__ double sm[];
    const long long t0 = wall_clock64();
    if (threadIdx.x == 0) sm[0] = 1.0;
    while (wall_clock64() - t0 < us * 100LL) __builtin_amdgcn_s_sleep(10);
    if (threadIdx.x == 0) { o[blockIdx.x] = cu_id(); t[2 * blockIdx.x] = t0; t[2 * blockIdx.x + 1] = wall_clock64(); }
}

int main() {
    hipDeviceProp_t pr;
    CK(hipGetDeviceProperties(&pr, 0));
    const int ncu = pr.multiProcessorCount;
    printf("CUs %d\n", ncu);
    const int words = (ncu + 31) / 32;
    unsigned *d;
    long long* dt;
    CK(hipMalloc(&d, 4 * 4096));
    CK(hipMalloc(&dt, 16 * 4096));
    std::vector<unsigned> h(4096);
    std::vector<long long> ht(2 * 4096);
    // 1) single-bit masks: where do bits 0..23 put a workgroup?
    for (int bit = 0; bit < 24; ++bit) {
        std::vector<uint32_t> m(words, 0u);
        m[bit / 32] = 1u << (bit % 32);
        hipStream_t s;
        if (hipExtStreamCreateWithCUMask(&s, words, m.data()) != hipSuccess) { printf("bit %d: create failed\n", bit); continue; }
        hipLaunchKernelGGL(k_hold, dim3(4), dim3(64), 0, s, d, dt, 5);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(h.data(), d, 16, hipMemcpyDeviceToHost));
        printf("bit %2d ->", bit);
        for (int i = 0; i < 4; ++i) printf(" x%u:%02x", h[i] >> 16, h[i] & 0xFF);
        printf("\n");
        CK(hipStreamDestroy(s));
    }
    // 2) heavy mask = bits [0, H), bulk mask = the rest; concurrent launches
    for (int H : {16, 32, 64}) {
        std::vector<uint32_t> mh(words, 0u), mb(words, 0u);
        for (int i = 0; i < ncu; ++i) (i < H ? mh : mb)[i / 32] |= 1u << (i % 32);
        hipStream_t sh, sb;
        CK(hipExtStreamCreateWithCUMask(&sh, words, mh.data()));
        CK(hipExtStreamCreateWithCUMask(&sb, words, mb.data()));
        const int GB = 2048, GH = H;
        hipLaunchKernelGGL(k_hold, dim3(GB), dim3(256), 70000, sb, d, dt, 50);
        hipLaunchKernelGGL(k_hold, dim3(GH), dim3(512), 120000, sh, d + GB, dt + 2 * GB, 200);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h.data(), d, 4 * (GB + GH), hipMemcpyDeviceToHost));
        CK(hipMemcpy(ht.data(), dt, 16 * (GB + GH), hipMemcpyDeviceToHost));
        std::set<unsigned> cb, ch;
        long long tmin = ht[0], hstart = 0, hend = 0, bend = 0;
        for (int i = 0; i < GB + GH; ++i) tmin = std::min(tmin, ht[2 * i]);
        for (int i = 0; i < GB; ++i) { cb.insert(h[i]); bend = std::max(bend, ht[2 * i + 1] - tmin); }
        for (int i = GB; i < GB + GH; ++i) { ch.insert(h[i]); hstart = std::max(hstart, ht[2 * i] - tmin); hend = std::max(hend, ht[2 * i + 1] - tmin); }
        int both = 0;
        for (unsigned c : ch) both += cb.count(c);
        std::map<unsigned, int> perx;
        for (unsigned c : ch) perx[c >> 16]++;
        printf("H=%d: bulk on %zu CUs, heavy on %zu CUs, shared %d; heavy last start %.1f us, heavy end %.1f us, bulk end %.1f us; heavy CUs per xcc:",
               H, cb.size(), ch.size(), both, hstart / 100.0, hend / 100.0, bend / 100.0);
        for (auto& kv : perx) printf(" %u:%d", kv.first, kv.second);
        printf("\n");
        CK(hipStreamDestroy(sh));
        CK(hipStreamDestroy(sb));
    }
    // 3) two-stream step hand-off: K steps of (bulk 20 us on A, heavy 20 us on B), each waiting
    // for the other's previous step, vs the same kernels back to back on one stream
    {
        hipStream_t a, b;
        CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
        CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
        hipEvent_t ea[2], eb[2], t0, t1;
        for (int i = 0; i < 2; ++i) { CK(hipEventCreateWithFlags(&ea[i], hipEventDisableTiming)); CK(hipEventCreateWithFlags(&eb[i], hipEventDisableTiming)); }
        CK(hipEventCreate(&t0));
        CK(hipEventCreate(&t1));
        const int K = 50;
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipEventRecord(t0, a));
            for (int k = 0; k < K; ++k) {
                if (k) CK(hipStreamWaitEvent(a, eb[(k - 1) & 1], 0));
                hipLaunchKernelGGL(k_hold, dim3(256), dim3(256), 0, a, d, dt, 20);
                CK(hipEventRecord(ea[k & 1], a));
                if (k) CK(hipStreamWaitEvent(b, ea[(k - 1) & 1], 0));
                hipLaunchKernelGGL(k_hold, dim3(16), dim3(512), 0, b, d + 256, dt + 512, 20);
                CK(hipEventRecord(eb[k & 1], b));
            }
            CK(hipStreamWaitEvent(a, eb[(K - 1) & 1], 0));
            CK(hipEventRecord(t1, a));
            CK(hipEventSynchronize(t1));
            float ms2;
            CK(hipEventElapsedTime(&ms2, t0, t1));
            CK(hipEventRecord(t0, a));
            for (int k = 0; k < K; ++k) hipLaunchKernelGGL(k_hold, dim3(256), dim3(256), 0, a, d, dt, 20);
            CK(hipEventRecord(t1, a));
            CK(hipEventSynchronize(t1));
            float ms1;
            CK(hipEventElapsedTime(&ms1, t0, t1));
            printf("step: two streams %.2f us, one stream %.2f us (kernel 20 us)\n", ms2 * 1e3 / K, ms1 * 1e3 / K);
        }
    }
    return 0;
}
