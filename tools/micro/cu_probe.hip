// CU identity probe (diagnostic): 512 co-resident workgroups (each holds its slot ~100 us)
// record HW_REG_HW_ID and HW_REG_XCC_ID; prints the distinct (xcc, hw_id field) values and
// how many workgroups share each, for several bit fields of HW_ID.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>
__global__ void k(unsigned* o) {
    const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
    const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11));
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < 10000) __builtin_amdgcn_s_sleep(10);  // ~100 us at 100 MHz
    if (threadIdx.x == 0) { o[2 * blockIdx.x] = hw; o[2 * blockIdx.x + 1] = xcc; }
}
int main() {
    const int G = 512;
    unsigned* d;
    (void)hipMalloc(&d, 8 * G);
    hipLaunchKernelGGL(k, dim3(G), dim3(256), 40000, 0, d);  // 40 KB LDS: at most 4 per CU
    std::vector<unsigned> h(2 * G);
    (void)hipMemcpy(h.data(), d, 8 * G, hipMemcpyDeviceToHost);
    for (int sh : {0, 8}) {
        for (int bits : {8, 12}) {
            std::map<unsigned, int> c;
            for (int b = 0; b < G; ++b) c[((h[2 * b + 1] & 15u) << 16) | ((h[2 * b] >> sh) & ((1u << bits) - 1))]++;
            std::map<int, int> mult;
            for (auto& kv : c) mult[kv.second]++;
            printf("HW_ID >> %d, %d bits: %zu distinct;", sh, bits, c.size());
            for (auto& kv : mult) printf(" %d x%d", kv.second, kv.first);
            printf("\n");
        }
    }
    for (int b = 0; b < 8; ++b) printf("wg %d: hw_id 0x%08x xcc 0x%x\n", b, h[2 * b], h[2 * b + 1]);
    return 0;
}
