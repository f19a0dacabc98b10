// solve_big.hip -- the ADMM kernel for long horizons (many factor blocks).
//
// Why a separate kernel: the 256-thread k_solve keeps the block-tridiagonal factor
// of K = P + sigma I + A' diag(rho) A in registers only up to 8 blocks; beyond that
// (NB = 0 instantiation) every ADMM iteration re-reads three 32 x 32 tiles per block
// from the per-instance workspace -- 3 * 17 * 8 KB = 408 KB per iteration at
// cfg 5 (N = 50, nb = 17), far more than an XCD's L2 holds for its resident
// instances, so the sweep ran at HBM speed (~55k cycles per iteration).
//
// Here one 512-thread workgroup (8 waves, two per SIMD) holds the whole factor on
// chip:
//   registers  S_k^{-1}[i][jl + 16 c] (c < 2) for every block k   (2 doubles / block)
//              H_k[i][jl] = F_{k+1}[jl][i]  (jl < amax <= 16)       (1 double / block)
//              with (i, jl) = (t / 16, t % 16): row i is summed by one 16-lane DPP row
//   LDS        F_k rows r < amax (the only nonzero rows: block k couples to block
//              k-1 through its first BFS level), amax x 32 per block
// and the sweep is
//   forward   k = 1..nb-1:  t_{k-1} = S_{k-1}^{-1} w_{k-1},  w_k -= F_k w_{k-1}   (1 barrier)
//             t_{nb-1} = S_{nb-1}^{-1} w_{nb-1}
//   backward  k = nb-2..0:  x_k = t_k - H_k x_{k+1}[0, amax)                     (1 barrier)
// -- the same elimination as solve.hip::bt_solve with the tiles on chip.
//
// Everything else (rhs gather, row update, termination checks, rho adaptation,
// refactorisation, unscaling) follows solve.hip's k_solve with 512 threads.
// Reference semantics: OSQP 0.6 osqp_solve (Control/MPC/mpc_dynamics.py:392-396 at
// N = 30 / 50); tests/test_gpu_parity.py and tests/test_mpc_device.py compare with
// the CPU oracle.
#include <hip/hip_runtime.h>

#include <cstring>
#include <type_traits>

#include "solve_phases.h"
#include "wave_util.h"

namespace mpcqp {

constexpr int TB = kThreadsBig;
// row stride of the F / G rows in LDS: 42 doubles.  The interface form's chain lanes (r, q)
// read row r, columns [8 q, 8 q + 8) as ds_read_b128, and the backward chain / fill lanes read
// the columns 4 q + c of row block k at row i: with a stride of 2 (mod 8) doubles both are
// conflict-free (LDS bank model, 64 banks of 4 B: 16 LDS cycles for the four 16-byte reads of
// a step at 34, 38, 42, ..., 64 at 40, 32, 48)
constexpr int FGS = 42;

// ---------------------------------------------------------------------------
// Two-sided ("twisted") block factorisation of K = tridiag(E_k, D_k, E_{k+1}'),
// meeting at block p = pmeet:
//   top     k = 0 .. p-1 :  S_k = D_k - F_k E_k'        F_k = E_k S_{k-1}^{-1}     (rows < amax)
//   bottom  k = nb-1 .. p+1: T_k = D_k - G_k E_{k+1}    G_k = E_{k+1}' T_{k+1}^{-1} (rows toff_k + [0, bmax))
//   middle  M = D_p - F_p E_p' - G_p E_{p+1}
// E_k has nonzero rows < amax (block k's first BFS level) and nonzero columns in
// toff_{k-1} + [0, bmax) (block k-1's last level), so F_k and G_k are thin and the
// Schur corrections touch an amax x amax / bmax x bmax corner only.  The two chains
// run in lock-step -- threads 0-255 the top, 256-511 the bottom, wave 0 and wave 4
// invert their tiles at the same time -- so the factorisation takes max(p, nb-1-p)+1
// steps instead of nb.  Stored: Sg[k] = S_k^{-1} / M^{-1} / T_k^{-1};  Fg[k] rows
// < amax = F_k (k = 1..p);  Hg[k] rows < bmax = G_k's tail rows (k = p..nb-2).
// X2: four scratch tiles besides SLds' three.  False on a non-positive pivot.
template <int TT, class KP>
__device__ __forceinline__ bool factorize2(const KP& p, SLds& L, double* __restrict__ X2, double rho,
                                           double* __restrict__ Fg, double* __restrict__ Hg,
                                           double* __restrict__ Sg) {
    constexpr int HT = TT / 2;      // threads per chain
    constexpr int NF = 16 * S / HT;  // per-thread F / G buffer (amax, bmax <= 16)
    const int tid = threadIdx.x, half = tid / HT, u = tid % HT;
    const int nb = p.nb, amax = p.amax, bmax = p.bmax, pm = p.pmeet, ntgt = p.ntgt;
    const int nst = max(pm, nb - 1 - pm);
    const int2* __restrict__ tt = (const int2*)p.tterm;
    double *SP = L.SP, *DK = L.DK, *EK = L.EK;                                   // top chain
    double *SP2 = X2, *DK2 = X2 + SS, *EK2 = X2 + 2 * SS, *EKp = X2 + 3 * SS;   // bottom chain
    bool ok = true;
#ifdef MPCQP_PHASE_PROF
    long long tf = clock64();
#define FPH(k) if (tid == 0) { const long long t_ = clock64(); L.pacc[k] += t_ - tf; tf = t_; }
#else
#define FPH(k)
#endif
    auto init = [&](int k, double* D, double* E, int t0, int stride) {
        for (int e = t0; e < SS; e += stride) {
            const int r = e >> 5;
            D[e] = e == r * (S + 1) ? (p.pad_var[k * S + r] >= 0 ? p.sigma : 1.0) : 0.0;
            E[e] = 0.0;
        }
    };
    // every target of block k has one owner: its terms are summed in plan order
    auto assemble = [&](int k, double* D, double* E, int t0, int stride) {
#pragma unroll 1
        for (int t = p.asm_blk_ptr[k] + t0; t < p.asm_blk_ptr[k + 1]; t += stride) {
            double acc = 0.0;
            const int tn = p.tcnt[__builtin_amdgcn_readfirstlane(t)];  // the wave's largest count
#pragma unroll 4
            for (int j = 0; j < tn; ++j) {
                const int2 w = tt[(long)j * ntgt + t];
                const int a = w.x & 0xFFFF, bb = (int)((unsigned)w.x >> 16), r = w.y;
                acc += r < 0 ? L.Pv[a] : rho_of(L.ct[r], rho) * L.Acsc[a] * L.Acsc[bb];
            }
            const int tg = p.asm_tgt[t];
            if (tg < SS) D[tg] += acc;
            else E[tg - SS] += acc;
        }
    };
    // F_k = E_k S_{k-1}^{-1} (rows < amax) -> f, Fg[k]
    auto top_f = [&](int k, double (&f)[NF]) {
        int nf = 0;
#pragma unroll 1
        for (int o = u; o < amax * S; o += HT, ++nf) {
            const int r = o >> 5, j = o & (S - 1);
            double sacc = 0.0;
#pragma unroll 8
            for (int l = 0; l < S; ++l) sacc += EK[r * S + l] * SP[l * S + j];
            f[nf & (NF - 1)] = sacc;
            Fg[(long)k * SS + o] = sacc;
        }
    };
    // G_k = E_{k+1}' T_{k+1}^{-1} on block k's tail rows (E_{k+1} in EKp, T^{-1} in SP2) -> g, Hg[k]
    auto bot_g = [&](int k, int toff, double (&g)[NF], int t0, int stride) {
        int ng = 0;
#pragma unroll 1
        for (int o = t0; o < bmax * S; o += stride, ++ng) {
            const int a = o >> 5, j = o & (S - 1);
            double sacc = 0.0;
#pragma unroll 1
            for (int r = 0; r < amax; ++r) sacc += EKp[r * S + toff + a] * SP2[r * S + j];
            g[ng & (NF - 1)] = sacc;
            Hg[(long)k * SS + o] = sacc;
        }
    };
    // D -= F E' on the amax x amax corner (F rows in SP, E in EK)
    auto top_corr = [&](double* D, int t0, int stride) {
#pragma unroll 1
        for (int o = t0; o < amax * amax; o += stride) {
            const int r = o / amax, c = o - r * amax;
            double sacc = 0.0;
#pragma unroll 8
            for (int l = 0; l < S; ++l) sacc += SP[r * S + l] * EK[c * S + l];
            D[r * S + c] -= sacc;
        }
    };
    // D -= G E_{k+1} on the bmax x bmax tail corner (G rows in SP2, E_{k+1} in EKp)
    auto bot_corr = [&](double* D, int toff, int t0, int stride) {
#pragma unroll 1
        for (int o = t0; o < bmax * bmax; o += stride) {
            const int a = o / bmax, c = o - a * bmax;
            double sacc = 0.0;
#pragma unroll 1
            for (int r = 0; r < amax; ++r) sacc += SP2[a * S + r] * EKp[r * S + toff + c];
            D[(toff + a) * S + toff + c] -= sacc;
        }
    };

#pragma unroll 1
    for (int s = 0; s < nst; ++s) {
        const int kt = s, kb = nb - 1 - s;
        const bool top = half == 0 && s < pm, bot = half == 1 && s < nb - 1 - pm;
        const int toffb = kb < nb - 1 ? p.toff[kb] : 0;
        if (top) init(kt, DK, EK, u, HT);
        if (bot) init(kb, DK2, EK2, u, HT);
        __syncthreads();
        if (top) assemble(kt, DK, EK, u, HT);
        if (bot) assemble(kb, DK2, EK2, u, HT);
        __syncthreads();
        FPH(8)
        double f[NF];
        if (top && kt > 0) top_f(kt, f);
        if (bot && kb < nb - 1) bot_g(kb, toffb, f, u, HT);
        __syncthreads();  // every read of S_{k-1}^{-1} / T_{k+1}^{-1} done
        {
            int nf = 0;
            if (top && kt > 0)
                for (int o = u; o < amax * S; o += HT, ++nf) SP[o] = f[nf & (NF - 1)];
            if (bot && kb < nb - 1)
                for (int o = u; o < bmax * S; o += HT, ++nf) SP2[o] = f[nf & (NF - 1)];
        }
        __syncthreads();
        if (top && kt > 0) top_corr(DK, u, HT);
        if (bot && kb < nb - 1) bot_corr(DK2, toffb, u, HT);
        __syncthreads();
        FPH(9)
        // wave 0 inverts the top tile, wave 4 the bottom one, at the same time
        double* okslot = EK + 2 * S;
        double* okslot2 = EKp + 2 * S;
        const bool topw = s < pm, botw = s < nb - 1 - pm;
        if (tid < 64 && topw) {
            const bool okw = gj_wave<true>(DK, EK, Sg + (long)kt * SS);
            if (tid == 0) okslot[0] = okw ? 1.0 : 0.0;
        }
        if (tid >= HT && tid < HT + 64 && botw) {
            const bool okw = gj_wave<true>(DK2, EKp, Sg + (long)kb * SS);
            if (tid == HT) okslot2[0] = okw ? 1.0 : 0.0;
        }
        __syncthreads();
        if (topw && !(okslot[0] > 0.5)) ok = false;
        if (botw && !(okslot2[0] > 0.5)) ok = false;
        FPH(10)
        if (topw) { double* t = SP; SP = DK; DK = t; }
        if (botw) {
            double* t = SP2; SP2 = DK2; DK2 = t;
            t = EKp; EKp = EK2; EK2 = t;  // E_kb is the next bottom step's E_{k+1}
        }
        __syncthreads();  // the okslots are rewritten by the next step's init
    }
    // middle block: both corrections, then its inverse
    {
        const int toffp = pm < nb - 1 ? p.toff[pm] : 0;
        init(pm, DK, EK, tid, TT);
        __syncthreads();
        assemble(pm, DK, EK, tid, TT);
        __syncthreads();
        FPH(8)
        double f[NF];
        if (half == 0 && pm > 0) top_f(pm, f);
        if (half == 1 && pm < nb - 1) bot_g(pm, toffp, f, u, HT);
        __syncthreads();
        {
            int nf = 0;
            if (half == 0 && pm > 0)
                for (int o = u; o < amax * S; o += HT, ++nf) SP[o] = f[nf & (NF - 1)];
            if (half == 1 && pm < nb - 1)
                for (int o = u; o < bmax * S; o += HT, ++nf) SP2[o] = f[nf & (NF - 1)];
        }
        __syncthreads();
        if (pm > 0) top_corr(DK, tid, TT);
        __syncthreads();
        if (pm < nb - 1) bot_corr(DK, toffp, tid, TT);
        __syncthreads();
        FPH(9)
        double* okslot = EK + 2 * S;
        if (tid < 64) {
            const bool okw = gj_wave<true>(DK, EK, Sg + (long)pm * SS);
            if (tid == 0) okslot[0] = okw ? 1.0 : 0.0;
        }
        __syncthreads();
        if (!(okslot[0] > 0.5)) ok = false;
        FPH(10)
    }
#undef FPH
    return ok;
}

// Gauss-Jordan of the rows in `piv` (bit r: row r; increasing order) of the tile T (row
// stride S; LDS or the workspace) by one wave, in place: gj_seg's rolled step with any row
// set.  Rows in `done` were pivoted before (the sign rule M_ij = -M_ji tells pivoted rows
// apart).  Before the first pivot, corrections are added to the unpivoted corners:
// dl[a * 16 + c] to T[o1 + a][o1 + c] (a, c < n1) and dl2 likewise at o2 / n2 (n = 0: none).
// Rows of T are loaded into registers once and stored back once.  False on a non-positive
// pivot.  buf: 2 S doubles of LDS.
__device__ __forceinline__ bool gj_rows(double* __restrict__ T, double* __restrict__ buf, const unsigned piv,
                                        const unsigned done, const double* __restrict__ dl, const int o1, const int n1,
                                        const double* __restrict__ dl2, const int o2, const int n2,
                                        double* __restrict__ T2 = nullptr) {
    const int lane = threadIdx.x & 63, i = lane & 31, h = lane >> 5;
    double v[16];
#pragma unroll
    for (int jj = 0; jj < 16; jj += 2) {
        const double2 t2 = *(const double2*)(T + i * S + 16 * h + jj);
        v[jj] = t2.x;
        v[jj + 1] = t2.y;
    }
    if (n1 > 0 && i >= o1 && i < o1 + n1) {
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
            const int c = 16 * h + jj - o1;
            if (c >= 0 && c < n1) v[jj] += dl[(i - o1) * 16 + c];
        }
    }
    if (n2 > 0 && i >= o2 && i < o2 + n2) {
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
            const int c = 16 * h + jj - o2;
            if (c >= 0 && c < n2) v[jj] += dl2[(i - o2) * 16 + c];
        }
    }
    double minpiv = 1.0, sc = 1.0, iv = 1.0;
    bool pivd = ((done >> i) & 1u) != 0;  // row i already pivoted
    int slot = 0;  // the publish buffer alternates between the pivots taken
    // unrolled over the 32 columns with a uniform skip of the rows not in `piv`: the pivot
    // column is a register index known at compile time (the rolled loop's scalar switch
    // picks, pick16 / put16, cost a multi-way branch twice per pivot)
#pragma unroll
    for (int p = 0; p < S; ++p) {
        if (!((piv >> p) & 1u)) continue;  // (uniform)
        const int pj = p & 15, ph = p >> 4;
        double* rb = buf + slot * S;
        slot ^= 1;
        if (h == ph) {
            const double vp = sc * v[pj];
            rb[i] = pivd ? -vp : vp;  // row p = +-column p
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const double pv = rb[p];
        const double mi = rb[i];
        double rowv[16];
#pragma unroll
        for (int jj = 0; jj < 16; jj += 2) {
            const double2 r2 = *(const double2*)(rb + 16 * h + jj);
            rowv[jj] = r2.x;
            rowv[jj + 1] = r2.y;
        }
        const double colv = pivd ? -mi : mi;
        minpiv = pv > 0.0 ? minpiv : -1.0;
        double d = __builtin_amdgcn_rcp(pv);
        d = __builtin_fma(d, __builtin_fma(-pv, d, 1.0), d);
        d = __builtin_fma(d, __builtin_fma(-pv, d, 1.0), d);
        const bool self = i == p;
        const double cd = self ? 0.0 : (colv * d) * iv;
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) v[jj] = __builtin_fma(-cd, rowv[jj], v[jj]);
        sc = self ? d : sc;
        iv = self ? pv : iv;
        if (h == ph) v[pj] = self ? 1.0 : -cd;
        pivd = pivd || self;
    }
#pragma unroll
    for (int jj = 0; jj < 16; jj += 2) *(double2*)(T + i * S + 16 * h + jj) = make_double2(sc * v[jj], sc * v[jj + 1]);
    if (T2)  // (a second copy: the LDS chain's workspace write-back)
#pragma unroll
        for (int jj = 0; jj < 16; jj += 2)
            *(double2*)(T2 + i * S + 16 * h + jj) = make_double2(sc * v[jj], sc * v[jj + 1]);
    return minpiv > 0.0;
}

// A barrier that orders LDS only: the chain's workspace stores (the write-back of S_k^{-1},
// F_k, G_k) are read by nothing before the factorisation's closing __syncthreads, so no barrier
// of the chain waits for them to land
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// factorize2s's chain with its operands in LDS (round 6).  In the workspace form every step
// waited on HBM / L2 round trips: the product read S_{k-1}^{-1} back from the workspace tile
// the previous step's pivots had just stored, the corner pivots loaded their tile from the
// workspace, and every __syncthreads after a workspace store waited for it to land.  Here
//   * the tile a step pivots (stage 1's S_k in the workspace) and the E_k coupling block of
//     the next step (amax x bmax of E_k, row stride 16) are loaded while the products run;
//   * the corner pivots run on the LDS tile and store the result twice: LDS (the next step's
//     S_{k-1}^{-1}) and the workspace (the solve's factor; never read back here);
//   * the barriers order LDS only (lds_barrier).
// Same sums in the same order on the same values: the factor is bit-identical to the
// workspace form's.  Xl: two tiles per chain (prev / current), two E blocks per chain.
template <int TT, class KP>
__device__ __forceinline__ bool factorize2s_lds_chain(const KP& p, SLds& L, double* __restrict__ Fg,
                                                      double* __restrict__ Hg, double* __restrict__ Sg,
                                                      double* __restrict__ Xl, const int ntop, const int nbot,
                                                      const int nst, bool okw) {
    constexpr int NW = TT / 64, HT = TT / 2;
    const int tid = threadIdx.x, w = tid >> 6, half = tid / HT, u = tid % HT;
    const int nb = p.nb, amax = p.amax, bmax = p.bmax, pm = p.pmeet;
#if defined(MPCQP_PHASE_PROF) && defined(MPCQP_CHAIN_STAMPS)
    long long tc = clock64();  // (diagnostic: wave 0's products / corners / pivots, slots 8 / 10 / 11)
#define CPH(k) if (tid == 0) { const long long t_ = clock64(); L.pacc[k] += t_ - tc; tc = t_; }
#else
#define CPH(k)
#endif
    double* const Fl = L.SP;
    double* const Gl = L.SP + 16 * S;
    double* const dlt = L.SP + 32 * S;
    double* const dlb = dlt + 256;
    double* const bufw = dlb + 256 + w * 2 * S;
    double* const tT = Xl;             // top tiles [2][SS]
    double* const tB = Xl + 2 * SS;    // bottom tiles [2][SS]
    double* const eT = Xl + 4 * SS;    // top E blocks [2][256]
    double* const eB = eT + 512;       // bottom E blocks [2][256]
    auto rows = [&](int a, int n) -> unsigned { return n <= 0 ? 0u : (((n >= 32 ? ~0u : ((1u << n) - 1u))) << a); };
    // the chains' blocks at step s (-1: none)
    auto top_k = [&](int s) { return s == nst + 1 ? (pm > 0 ? pm : -1) : (s <= ntop ? s : -1); };
    auto bot_k = [&](int s) { return s == nst + 1 ? (pm < nb - 1 ? pm : -1) : (s <= nbot ? nb - 1 - s : -1); };
    // E block of step s: element i of the half's 256 (row i / 16, column i % 16)
    constexpr int NE = 256 / HT;
    auto e_load = [&](int s, int i) -> double {
        const int r = i >> 4, c = i & 15;
        if (half == 0) {
            const int kt = top_k(s);
            if (kt < 0 || r >= amax || c >= bmax) return 0.0;
            return Fg[(long)kt * SS + r * S + p.toff[kt - 1] + c];
        }
        const int kb = bot_k(s);
        if (kb < 0 || r >= amax || c >= bmax) return 0.0;
        return Fg[(long)(kb + 1) * SS + r * S + p.toff[kb] + c];
    };
    // chain start: the end blocks' inverses (stage 1) as the first steps' S_{k-1}^{-1} / T_{k+1}^{-1},
    // and the first step's E blocks
    {
        const double* src = half == 0 ? Sg : Sg + (long)(nb - 1) * SS;
        double* dst = half == 0 ? tT : tB;
        for (int e = 2 * u; e < SS; e += 2 * HT) *(double2*)(dst + e) = *(const double2*)(src + e);
#pragma unroll
        for (int q = 0; q < NE; ++q) (half == 0 ? eT : eB)[u + q * HT] = e_load(1, u + q * HT);
    }
    lds_barrier();
    int pT = 0, pB = 0, qe = 0;  // prev tile of each chain, current E block
#pragma unroll 1
    for (int s = 1; s <= nst + 1; ++s) {
        const bool mid = s == nst + 1;
        const int kt = mid ? pm : s, kb = mid ? pm : nb - 1 - s;
        const bool top = mid ? pm > 0 : s <= ntop;
        const bool bot = mid ? pm < nb - 1 : s <= nbot;
        // this step's tile (stage 1's S_k in the workspace): the top half loads the top (or
        // middle) block, the bottom half the bottom one -- in flight under the products
        const bool ldt = half == 0 ? (top || mid) : (bot && !mid);
        const double* tsrc = Sg + (long)(half == 0 ? kt : kb) * SS;
        double2 tv[SS / (2 * HT)];
#pragma unroll
        for (int q = 0; q < SS / (2 * HT); ++q)
            tv[q] = ldt ? *(const double2*)(tsrc + 2 * u + q * 2 * HT) : make_double2(0.0, 0.0);
        double en[NE];  // the next step's E block
#pragma unroll
        for (int q = 0; q < NE; ++q) en[q] = s <= nst ? e_load(s + 1, u + q * HT) : 0.0;
        const double* Et = eT + qe * 256;
        const double* Eb = eB + qe * 256;
        // products: F_kt (top half's threads), G_kb (bottom half's)
        if (half == 0 && top) {
            const double* Sp = tT + pT * SS;
            const int l0 = p.toff[kt - 1];
            for (int o = u; o < amax * S; o += HT) {
                const int r = o >> 5, j = o & (S - 1);
                double sacc = 0.0;
                for (int l = 0; l < bmax; ++l) sacc += Et[r * 16 + l] * Sp[(l0 + l) * S + j];
                Fl[o] = sacc;
            }
        }
        if (half == 1 && bot) {
            const double* Tn = tB + pB * SS;
            for (int o = u; o < bmax * S; o += HT) {
                const int a = o >> 5, j = o & (S - 1);
                double sacc = 0.0;
                for (int r = 0; r < amax; ++r) sacc += Eb[r * 16 + a] * Tn[r * S + j];
                Gl[o] = sacc;
            }
        }
        {
            double* td = (half == 0 ? tT + (pT ^ 1) * SS : tB + (pB ^ 1) * SS);
            if (ldt)
#pragma unroll
                for (int q = 0; q < SS / (2 * HT); ++q) *(double2*)(td + 2 * u + q * 2 * HT) = tv[q];
#pragma unroll
            for (int q = 0; q < NE; ++q) (half == 0 ? eT : eB)[(qe ^ 1) * 256 + u + q * HT] = en[q];
        }
        lds_barrier();
        CPH(8)
        // corners: -F E' (amax x amax), -G E_{kb+1} (bmax x bmax); F -> Fg[kt], G -> Hg[kb]
        if (half == 0 && top) {
            if (u < amax * amax) {
                const int r = u / amax, c = u - r * amax;
                double sacc = 0.0;
                for (int l = 0; l < bmax; ++l) sacc += Fl[r * S + p.toff[kt - 1] + l] * Et[c * 16 + l];
                dlt[r * 16 + c] = -sacc;
            }
            for (int o = u; o < amax * S; o += HT) Fg[(long)kt * SS + o] = Fl[o];
        }
        if (half == 1 && bot) {
            if (u < bmax * bmax) {
                const int a = u / bmax, c = u - a * bmax;
                double sacc = 0.0;
                for (int r = 0; r < amax; ++r) sacc += Gl[a * S + r] * Eb[r * 16 + c];
                dlb[a * 16 + c] = -sacc;
            }
            for (int o = u; o < bmax * S; o += HT) Hg[(long)kb * SS + o] = Gl[o];
        }
        lds_barrier();
        CPH(10)
        // corner pivots on the LDS tiles: wave 0 the top (or middle) block, wave NW/2 + 1 the bottom one
        if (mid) {
            if (w == 0) {
                const unsigned ct = top ? rows(0, amax) : 0u;
                const unsigned cb = bot ? rows(p.toff[pm], bmax) : 0u;
                const unsigned all = rows(0, p.bsize[pm]);
                okw = gj_rows(tT + (pT ^ 1) * SS, bufw, (ct | cb) & all, all & ~(ct | cb), dlt, 0, top ? amax : 0,
                              dlb, bot ? p.toff[pm] : 0, bot ? bmax : 0, Sg + (long)pm * SS) && okw;
            }
        } else {
            if (w == 0 && top) {
                const unsigned c = rows(0, amax), all = rows(0, p.bsize[kt]);
                okw = gj_rows(tT + (pT ^ 1) * SS, bufw, c & all, all & ~c, dlt, 0, amax, nullptr, 0, 0,
                              Sg + (long)kt * SS) && okw;
            }
            // (wave NW/2 + 1: the top chain's wave 0 and wave NW/2 share a SIMD -- the two
            // pivot chains would interleave on one VALU)
            if (w == NW / 2 + 1 && bot) {
                const unsigned c = rows(p.toff[kb], bmax), all = rows(0, p.bsize[kb]);
                okw = gj_rows(tB + (pB ^ 1) * SS, bufw, c & all, all & ~c, nullptr, 0, 0, dlb, p.toff[kb], bmax,
                              Sg + (long)kb * SS) && okw;
            }
        }
        lds_barrier();
        CPH(11)
        if (top) pT ^= 1;
        if (bot && !mid) pB ^= 1;
        qe ^= 1;
    }
    #undef CPH
    return okw;
}

// The two-sided factorisation split like factorize_g (round 4): the Gauss-Jordan pivots that
// do not wait for a neighbouring block come off the chain.  S_k (top), T_k (bottom) and M
// (middle) differ from the assembled D_k only on the coupling corners -- rows [0, amax) for a
// top block's link to block k-1, rows [toff_k, toff_k + bmax) for a bottom block's link to
// block k+1, both for the middle -- so:
//   stage 1, the eight waves over the blocks (wave w: k = w, w + 8, ...): fill D_k (zeros,
//     the diagonal) in the workspace tile Sg[k] and E_k (rows < amax) in Fg[k], write every
//     assembly target once, and pivot every row of D_k outside its corners (blocks 0 and
//     nb-1 whole);
//   the chain, both ends in lock-step: top k = 1 .. p-1: F_k = E_k S_{k-1}^{-1} over E_k's
//     nonzero columns (LDS, then Fg[k]), the corner -F_k E_k', wave 0 pivots rows [0, amax);
//     bottom k = nb-2 .. p+1: G_k = E_{k+1}[:, toff_k + .]' T_{k+1}^{-1}[0, amax) (LDS, then
//     Hg[k]), the corner -G_k E_{k+1}, wave 4 pivots the tail rows;
//   the middle: both products and corners, wave 0 pivots both row sets.
// The chain's Gauss-Jordan is amax (bmax) pivots a step instead of 32, and stage 1 runs on
// eight waves at once.  Same outputs as factorize2 (Sg: S_k^{-1} / M^{-1} / T_k^{-1}; Fg rows
// < amax: F_k, k = 1..p; Hg rows < bmax: G_k, k = p..nb-2); the inverses agree at rounding
// level (the pivot order differs).  Scratch: the LDS tiles of SLds (SP, DK, EK).
// Xl (or null): the LDS chain (factorize2s_lds_chain) -- 4 S x S + 1024 doubles of scratch.
template <int TT, class KP>
__device__ __forceinline__ bool factorize2s(const KP& p, SLds& L, double rho, double* __restrict__ Fg,
                                            double* __restrict__ Hg, double* __restrict__ Sg,
                                            double* __restrict__ Xl = nullptr) {
    constexpr int NW = TT / 64, HT = TT / 2;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, half = tid / HT, u = tid % HT;
    const int nb = p.nb, amax = p.amax, bmax = p.bmax, pm = p.pmeet;
    double* const Fl = L.SP;                   // F_k of the top step, amax x 32
    double* const Gl = L.SP + 16 * S;          // G_k of the bottom step, bmax x 32
    double* const dlt = L.SP + 32 * S;         // top corner correction, row stride 16
    double* const dlb = dlt + 256;             // bottom corner correction
    double* const bufw = dlb + 256 + w * 2 * S;
    double* const okf = bufw + (NW - w) * 2 * S;  // NW flags after the buffers
    auto gsync = []() __attribute__((always_inline)) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    };
    auto rows = [&](int a, int n) -> unsigned { return n <= 0 ? 0u : (((n >= 32 ? ~0u : ((1u << n) - 1u))) << a); };
#ifdef MPCQP_PHASE_PROF
    long long tf = clock64();
#define FPH(k) if (tid == 0) { const long long t_ = clock64(); L.pacc[k] += t_ - tf; tf = t_; }
#else
#define FPH(k)
#endif
    bool okw = true;
    // stage 1
#pragma unroll 1
    for (int k = w; k < nb; k += NW) {
        double* D = Sg + (long)k * SS;
        double* E = Fg + (long)k * SS;
        for (int e = 2 * lane; e < SS; e += 128) {
            const int r = e >> 5, c = e & (S - 1);  // c even: the diagonal is (r, r)
            const double dg = p.pad_var[k * S + r] >= 0 ? p.sigma : 1.0;
            *(double2*)(D + e) = make_double2(c == r ? dg : 0.0, c + 1 == r ? dg : 0.0);
        }
        if (k > 0)
            for (int e = 2 * lane; e < amax * S; e += 128) *(double2*)(E + e) = make_double2(0.0, 0.0);
        gsync();
        assemble_targets<false, false, true>(p, L, rho, k, D, E, lane, 64);
        gsync();
#ifndef MPCQP_CHAIN_STAMPS
        FPH(8)
#endif
        unsigned cut = 0;
        if (k > 0 && k <= pm) cut |= rows(0, amax);              // the link to block k-1
        if (k < nb - 1 && k >= pm) cut |= rows(p.toff[k], bmax);  // the link to block k+1
        const unsigned all = rows(0, p.bsize[k]);
        okw = gj_rows(D, bufw, all & ~cut, 0u, nullptr, 0, 0, nullptr, 0, 0) && okw;
#ifndef MPCQP_CHAIN_STAMPS
        FPH(10)
#endif
    }
    __syncthreads();
#ifndef MPCQP_CHAIN_STAMPS
    FPH(11)
#endif
    const int ntop = pm - 1 > 0 ? pm - 1 : 0, nbot = nb - 2 - pm > 0 ? nb - 2 - pm : 0;
    const int nst = ntop > nbot ? ntop : nbot;
    if (Xl) {
        okw = factorize2s_lds_chain<TT>(p, L, Fg, Hg, Sg, Xl, ntop, nbot, nst, okw);
        FPH(9)
    } else {
    // step s: top block kt = s (s <= ntop), bottom block kb = nb - 1 - s (s <= nbot); s = nst + 1:
    // the middle block (both links)
#pragma unroll 1
    for (int s = 1; s <= nst + 1; ++s) {
        const bool mid = s == nst + 1;
        const int kt = mid ? pm : s, kb = mid ? pm : nb - 1 - s;
        const bool top = mid ? pm > 0 : s <= ntop;
        const bool bot = mid ? pm < nb - 1 : s <= nbot;
        // products: F_kt (top half's threads), G_kb (bottom half's)
        if (half == 0 && top) {
            const double* Sp = Sg + (long)(kt - 1) * SS;
            const double* E = Fg + (long)kt * SS;
            const int l0 = p.toff[kt - 1];
            for (int o = u; o < amax * S; o += HT) {
                const int r = o >> 5, j = o & (S - 1);
                double sacc = 0.0;
                for (int l = l0; l < l0 + bmax; ++l) sacc += E[r * S + l] * Sp[l * S + j];
                Fl[o] = sacc;
            }
        }
        if (half == 1 && bot) {
            const double* Tn = Sg + (long)(kb + 1) * SS;
            const double* E = Fg + (long)(kb + 1) * SS;
            const int to = p.toff[kb];
            for (int o = u; o < bmax * S; o += HT) {
                const int a = o >> 5, j = o & (S - 1);
                double sacc = 0.0;
                for (int r = 0; r < amax; ++r) sacc += E[r * S + to + a] * Tn[r * S + j];
                Gl[o] = sacc;
            }
        }
        __syncthreads();
        // corners: -F E' (amax x amax), -G E_{kb+1} (bmax x bmax); F -> Fg[kt], G -> Hg[kb]
        if (half == 0 && top) {
            const double* E = Fg + (long)kt * SS;
            const int l0 = p.toff[kt - 1];
            if (u < amax * amax) {
                const int r = u / amax, c = u - r * amax;
                double sacc = 0.0;
                for (int l = l0; l < l0 + bmax; ++l) sacc += Fl[r * S + l] * E[c * S + l];
                dlt[r * 16 + c] = -sacc;
            }
        }
        if (half == 1 && bot) {
            const double* E = Fg + (long)(kb + 1) * SS;
            const int to = p.toff[kb];
            if (u < bmax * bmax) {
                const int a = u / bmax, c = u - a * bmax;
                double sacc = 0.0;
                for (int r = 0; r < amax; ++r) sacc += Gl[a * S + r] * E[r * S + to + c];
                dlb[a * 16 + c] = -sacc;
            }
            for (int o = u; o < bmax * S; o += HT) Hg[(long)kb * SS + o] = Gl[o];
        }
        __syncthreads();  // (E_kt's reads are done: F_kt may overwrite it in Fg[kt])
        if (half == 0 && top)
            for (int o = u; o < amax * S; o += HT) Fg[(long)kt * SS + o] = Fl[o];
        FPH(9)
        // corner pivots: wave 0 the top (or middle) block, wave NW/2 the bottom one
        if (mid) {
            if (w == 0) {
                const unsigned ct = top ? rows(0, amax) : 0u;
                const unsigned cb = bot ? rows(p.toff[pm], bmax) : 0u;
                const unsigned all = rows(0, p.bsize[pm]);
                okw = gj_rows(Sg + (long)pm * SS, bufw, (ct | cb) & all, all & ~(ct | cb), dlt, 0, top ? amax : 0,
                              dlb, bot ? p.toff[pm] : 0, bot ? bmax : 0) && okw;
            }
        } else {
            if (w == 0 && top) {
                const unsigned c = rows(0, amax), all = rows(0, p.bsize[kt]);
                okw = gj_rows(Sg + (long)kt * SS, bufw, c & all, all & ~c, dlt, 0, amax, nullptr, 0, 0) && okw;
            }
            if (w == NW / 2 && bot) {
                const unsigned c = rows(p.toff[kb], bmax), all = rows(0, p.bsize[kb]);
                okw = gj_rows(Sg + (long)kb * SS, bufw, c & all, all & ~c, nullptr, 0, 0, dlb, p.toff[kb], bmax) && okw;
            }
        }
        __syncthreads();
        FPH(11)
    }
    }
#undef FPH
    if (lane == 0) okf[w] = okw ? 1.0 : 0.0;
    __syncthreads();
    bool ok = true;
#pragma unroll
    for (int k = 0; k < NW; ++k) ok = ok && okf[k] > 0.5;
    __syncthreads();  // (the flags are read before any later reuse of the scratch)
    return ok;
}

// LDS after the common carve (solve.hip::lds_solve_bytes): the F rows
// (derived from the LDS carve by pointer arithmetic only, so the compiler keeps
// LDS instructions for it -- an integer round trip would make it a flat pointer)
__device__ __forceinline__ double* big_fc(const SLds& L) {
    char* c = (char*)(L.flag + 16);
    c += (16u - ((unsigned)(unsigned long)c & 15u)) & 15u;
    return A16((double*)c);
}

// the LDS chain's scratch (factorize2s_lds_chain) fits in the F / G region X2 (big_fg_len)
template <class KP>
__host__ __device__ inline int big_fg_len(const KP& p);
template <class KP>
__device__ __forceinline__ bool lds_chain_fits(const KP& p) {
    return p.lchain && p.amax <= 16 && p.bmax <= 16 && big_fg_len(p) >= 4 * SS + 1024;
}

template <int TT, class KP>
__device__ __noinline__ bool factorize2_nl(const KP* gp, long b, double rho, double* X2) {
    const KPc& p = kconst(gp);
    SL2 C = carve(p);
    bool ok;
    if constexpr (TT >= 256)  // (the two-wave variant 14 keeps the unsplit form)
        // (the F / G region from the carve, not the X2 argument: an LDS-typed pointer, so the
        // chain's tile and E accesses are ds_ instructions -- flat ones wait on the vector-memory
        // counter too, i.e. for the chain's own workspace loads and write-back stores)
        ok = factorize2s<TT>(p, C.L, rho, p.F + b * (long)p.nb * SS, p.H + b * (long)p.nb * SS,
                             p.Si + b * (long)p.nb * SS, lds_chain_fits(p) ? big_fc(C.L) : nullptr);
    else
        ok = factorize2<TT>(p, C.L, X2, rho, p.F + b * (long)p.nb * SS, p.H + b * (long)p.nb * SS,
                            p.Si + b * (long)p.nb * SS);
    // the rho the workspace factor belongs to (scal[3]), beside it: a solve reuses the factor only
    // when it is also the instance's current rho (scal[2]), whatever cleared or forgot ffresh
    if (threadIdx.x == 0) p.scal[b * 4 + 3] = ok ? rho : -1.0;
    return ok;
}

// The factor on chip for the two-sided sweep.  Thread t: half h = t / 256 (0 top,
// 1 bottom), (i, jg) = (t % 256 / 8, t % 8): row i of a tile is summed by one 8-lane
// DPP half-row, lane jg holding columns jg + 8c.
//   top    Inv[s] = S_s^{-1} (s < p), M^{-1} (s = SL-1)   (registers)
//   bottom Inv[s] = T_{nb-1-s}^{-1}                       (registers)
//   F_k rows (k = 1..p) and G_k tail rows (k = p..nb-2)  (LDS; the backward sweep
//   reads them transposed: H_k = F_{k+1}', T_k^{-1} E_k = G_{k-1}')
template <int SL>
struct TwoSided {
    double Inv[SL][4];
    // frows: also copy the F / G rows into LDS (after a factorisation, which uses that region as
    // scratch; a termination check leaves it alone, so a run start after one need not)
    __device__ __forceinline__ void load(int nb, int pm, int amax, int bmax, const double* __restrict__ Fg,
                                         const double* __restrict__ Hg, const double* __restrict__ Sg,
                                         double* __restrict__ Fc, double* __restrict__ Gc, bool frows) {
        const int tid = threadIdx.x, half = __builtin_amdgcn_readfirstlane(tid >> 8), u = tid & 255, i = u >> 3,
                  jg = u & 7;
        const int nbot = nb - 1 - pm;
#pragma unroll
        for (int s = 0; s < SL; ++s) {
            // top: S_s^{-1} in slot s < p, M^{-1} in the last slot (the middle step's operand at a
            // fixed place, not picked by p at run time); bottom: T_{nb-1-s}^{-1} in slot s < nb-1-p
            const bool have = half == 0 ? (s < pm || s == SL - 1) : s < nbot;
            const int k = half == 0 ? (s == SL - 1 ? pm : s) : nb - 1 - s;
#pragma unroll
            for (int c = 0; c < 4; ++c) Inv[s][c] = have ? Sg[(long)k * SS + i * S + jg + 8 * c] : 0.0;
        }
        if (!frows) return;
        for (int o = tid; o < pm * amax * S; o += TB) {  // row q = k amax + r of F_{k+1}
            const int q = o >> 5, j = o & (S - 1), k = q / amax, r = q - k * amax;
            Fc[q * FGS + j] = Fg[(long)(k + 1) * SS + r * S + j];
        }
        for (int o = tid; o < nbot * bmax * S; o += TB) {
            const int q = o >> 5, j = o & (S - 1), k = q / bmax, r = q - k * bmax;
            Gc[q * FGS + j] = Hg[(long)(pm + k) * SS + r * S + j];
        }
    }
};

__device__ __forceinline__ double dot4f(const double (&a)[4], const double (&v)[4]) {  // one mul, three fma
    return __builtin_fma(a[3], v[3], __builtin_fma(a[2], v[2], __builtin_fma(a[1], v[1], a[0] * v[0])));
}
__device__ __forceinline__ double dot4fn(const double (&a)[4], const double (&v)[4]) {  // -dot4f, exactly
    return __builtin_fma(-a[3], v[3], __builtin_fma(-a[2], v[2], __builtin_fma(-a[1], v[1], -a[0] * v[0])));
}
__device__ __forceinline__ double dot4c(const double (&a)[4], const double (&v)[4]) {
    return (a[0] * v[0] + a[1] * v[1]) + (a[2] * v[2] + a[3] * v[3]);
}

// xt = K^{-1} rb.  The forward sweeps' low-rank updates go into rb in place (the
// writer lane of a row reads the old value at the start of the step, off the critical
// path), except the bottom chain's update of the middle block, which the top chain
// updates too: it goes (negated) to corB[p][toff_p + a] (a < bmax), zero everywhere else (cleared
// once per solve, the same entries rewritten every iteration).  A step reads only its
// block of rb and the F / G row (8 LDS reads per lane, 16 before), sums two 8-lane DPP
// dot products side by side.  Both halves run the same instruction stream with per-half
// operands.  2 max(p, nb-1-p) + 1 barriers.  Same sums as the earlier read-only form
// (w - corT - corB), which subtracted exact zeros for the other chain.
// The LDS offsets of each step (twisted_solve), formed once per run instead of per step:
// bits 0-15 the forward step's destination row offset kd S (+ toff_kd on the bottom chain),
// bits 16-31 the backward step's x_{k+-1} offset.  Formed per step they were a dependent LDS
// read (toff) in front of the step's own reads.
// fo: the F / G row block of each step, in rows of the F / G region (FGS doubles): bits 0-15
// the forward step's F_s (top) / G_kd (bottom), bits 16-31 the backward step's H_k.
// All four are double offsets from the dynamic LDS base (sm), so a step forms its addresses
// from registers alone (no reload of a spilled base pointer in front of its reads):
//   so: bits 0-15 the forward step's destination row (rb or corB, + kd S + toff), bits 16-31
//       the backward step's x_{k+-1} (xt + ...);  fo: the F / G rows of the forward step,
//       bits 16-31 the backward step's H rows.
// The bottom chain's update of the middle block touches rows [toff_p, toff_p + bmax), the top
// chain's rows [0, amax): when those are disjoint (toff_p >= amax: the middle block's first and
// last BFS levels apart, every long-horizon workload here) the bottom chain updates rb in place
// like every other step, and the middle step reads w_p alone (no corB reads or subtraction).
template <class KP>
__device__ __forceinline__ int middle_apart(const KP& p, const int* toffL) {
    return p.apart && p.pmeet < p.nb - 1 && toffL[p.pmeet] >= p.amax;
}

template <int SL, int TT = 512, class KP>
__device__ __forceinline__ void step_offsets(const KP& p, const int* toffL, const double* rb, const double* xt,
                                             const double* corB, const double* Fc, int (&so)[SL], int (&fo)[SL]) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    const int half = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / (TT / 2)));
    const int nb = p.nb, pm = p.pmeet, nmine = half ? nb - 1 - pm : pm;
    const int amax = p.amax, bmax = p.bmax, g0 = pm * amax;  // (Gc = Fc + g0 FGS)
    const int orb = (int)(rb - sm), oxt = (int)(xt - sm), ocb = (int)(corB - sm), ofc = (int)(Fc - sm);
    const int apart = middle_apart(p, toffL);
#pragma unroll
    for (int s = 0; s < SL; ++s) {
        int f = 0, bk = 0, ff = 0, fb = 0;
        if (s >= 1 && s <= nmine) {
            const int kd = half ? nb - 1 - s : s;
            f = (half && kd == pm && !apart ? ocb : orb) + kd * S + (half ? toffL[kd] : 0);
            const int k = half ? pm + s : pm - s;
            bk = oxt + (half ? (k - 1) * S + toffL[k - 1] : (k + 1) * S);
            ff = ofc + (half ? g0 + (kd - pm) * bmax : (s - 1) * amax) * FGS;
            fb = ofc + (half ? g0 + (k - 1 - pm) * bmax : k * amax) * FGS;
        }
        so[s] = s == 0 ? apart : f | (bk << 16);  // (so[0]: no step; it carries middle_apart)
        fo[s] = ff | (fb << 16);
        asm volatile("" : "+v"(so[s]), "+v"(fo[s]));  // (in VGPRs: the kernel's scalar registers are spoken for)
    }
}

template <int SL, class KP>
__device__ __forceinline__ void twisted_solve(const TwoSided<SL>& R, const KP& p, const double* Fc,
                                              const double* Gc, const int* toffL, const int (&so)[SL],
                                              const int (&fo)[SL], double* rb, double* xt, double* corB,
                                              long long* pacc) {
    // PRE: the step offsets were formed at the run start (step_offsets); the long instantiation
    // (nb <= 24) has no registers for them and forms them per step
    constexpr bool PRE = SL <= 10;
    extern __shared__ __attribute__((aligned(16))) double sm[];
#ifdef MPCQP_PHASE_PROF
    long long t0s = clock64();
#define SPH(k) if (pacc && threadIdx.x == 0) { const long long t_ = clock64(); pacc[k] += t_ - t0s; t0s = t_; }
#else
#define SPH(k)
#endif
    int opq = 0;
    asm volatile("" : "+s"(opq));  // keep per-block LDS addresses out of the register budget
    const int tid = threadIdx.x, half = __builtin_amdgcn_readfirstlane(tid >> 8), u = tid & 255, i = u >> 3,
              jg = (u & 7) + opq, j0 = u & 7;
    const int nb = p.nb, pm = p.pmeet, amax = p.amax, bmax = p.bmax, nbot = nb - 1 - pm;
    int nst = nbot > pm ? nbot : pm, nmine = half ? nbot : pm;
    // (through an empty asm each call: the steps' tests against them stay scalar compares in
    // the loop -- hoisted out of the ADMM loop they were 64-bit masks spilled to VGPR lanes,
    // read back with v_readlane on every step)
    int nbo = nb, apart = __builtin_amdgcn_readfirstlane(PRE ? so[0] : middle_apart(p, toffL));
    asm volatile("" : "+s"(nst), "+s"(nmine), "+s"(nbo), "+s"(apart));
    const int lim = half ? bmax : amax;
    const bool writer = j0 == 0, lowrank = i < lim;
    const int ir = lowrank ? i : 0;  // F / G row this thread sums (row 0 for the rest: reads stay in range)
    // forward: top step s: t_{s-1} = S_{s-1}^{-1} w_{s-1}, w_s -= F_s w_{s-1};
    //          bottom step s (k = nb-1-s): t~_{k+1} = T_{k+1}^{-1} w~_{k+1}, w~_k -= G_k w~_{k+1}
#pragma unroll
    for (int s = 1; s < SL; ++s) {
        if (s <= nst) {
            if (s <= nmine) {
                const int ks = half ? nbo - s : s - 1, kd = half ? nb - 1 - s : s;
                const int woff = PRE ? 0 : kd * S + (half ? toffL[kd] : 0);
                const bool mid = half && s == nmine && !apart;  // (kd == pm: the bottom chain's last step)
                double* dst = PRE ? sm + (so[s] & 0xFFFF) + i : (mid ? corB : rb) + woff + i;
                const double old = *dst;  // (every lane: an unconditional read, the unused ones ignored)
                const double* w = rb + ks * S;
                const double v4[4] = {w[jg], w[jg + 8], w[jg + 16], w[jg + 24]};
                const double* f = PRE ? sm + (fo[s] & 0xFFFF) + ir * FGS
                                           : (half ? Gc + (kd - pm) * bmax * FGS : Fc + (s - 1) * amax * FGS) + ir * FGS;
                const double f4[4] = {f[jg], f[jg + 8], f[jg + 16], f[jg + 24]};
                // the two 8-lane sums paired: the first level (row_half_mirror, lane l with 7-l)
                // leaves lanes 0-3 summing the S^-1 row and lanes 4-7 the F row, so each later
                // level moves one double instead of two; lane 0 stores t and lane 4 the update,
                // in one store instruction
                int jo = j0;
                asm volatile("" : "+v"(jo));  // (the half-row split as a compare, not a spilled mask)
                const bool up = jo >= 4, sub = up && !mid;
                // the store's address and the value it adds to (o: the old value of an update,
                // 0 for t and for the middle block's correction) settled before the sums.  The
                // F row's products are summed negated (-c: the sign folded into the fma
                // operands, exact), so every store is o + sum -- t, old - c, or -c into corB
                // (the middle step adds it)
                __attribute__((address_space(3))) double* a =
                    (__attribute__((address_space(3))) double*)(up ? dst : xt + ks * S + i);
                double o = sub ? old : 0.0;
                asm volatile("" : "+v"(a), "+v"(o));
                const double tp = dot4f(R.Inv[s - 1], v4), cp = dot4fn(f4, v4);
                double x = up ? cp : tp;
                x += dpp<0x141>(up ? tp : cp);
                x += dpp<0xB1>(x);
                // the last level's add folded into the store: o + (x + y) as (o + x) + y, the
                // first add taken while y moves
                double pre = o + x;
                asm volatile("" : "+v"(pre));  // (kept out of the store's branch)
                const double y = dpp<0x4E>(x);
                if (writer || (j0 == 4 && lowrank)) *a = pre + y;
            }
            __syncthreads();
        }
    }
    SPH(12)
    // middle: x_p = M^{-1} w_p with both chains' corrections, by the top half
    if (half == 0) {
        const double* w = rb + pm * S;
        const double* cb = corB + pm * S;
        double v4[4];
        if (apart) {
#pragma unroll
            for (int c = 0; c < 4; ++c) v4[c] = w[jg + 8 * c];
        } else {  // (corB holds -c: twisted_solve's forward step)
#pragma unroll
            for (int c = 0; c < 4; ++c) v4[c] = w[jg + 8 * c] + cb[jg + 8 * c];
        }
        const double t = reduce8(dot4c(R.Inv[SL - 1], v4));  // (M^{-1}: TwoSided::load's last slot)
        if (writer) xt[pm * S + i] = t;
    }
    __syncthreads();
    SPH(13)
    // backward: top x_k = t_k - H_k x_{k+1}[0, amax) (k = p-1 .. 0);
    //           bottom x_k = t~_k - G_{k-1}' x_{k-1}[toff_{k-1} + (0, bmax)] (k = p+1 .. nb-1)
#pragma unroll
    for (int s = 1; s < SL; ++s) {
        if (s <= nst) {
            if (s <= nmine) {
                const int k = half ? pm + s : pm - s;
                const double* x1 = PRE ? sm + (so[s] >> 16) : xt + (half ? (k - 1) * S + toffL[k - 1] : (k + 1) * S);
                // H_k[i][r] = F_{k+1}[r][i] (top), G_{k-1}[r][i] (bottom); rows >= lim read as 0
                const double* h = PRE ? sm + (fo[s] >> 16) + i
                                           : (half ? Gc + (k - 1 - pm) * bmax * FGS : Fc + k * amax * FGS) + i;
                const double tk = xt[k * S + i];
                const int r0 = j0 < lim ? j0 : 0, r1 = j0 + 8 < lim ? j0 + 8 : 0;
                const double h0 = h[r0 * FGS], h1 = h[r1 * FGS], x0 = x1[r0], x8 = x1[r1];
                const double a0 = j0 < lim ? h0 * x0 : 0.0;
                const double a1 = j0 + 8 < lim ? h1 * x8 : 0.0;
                double c = a0 + a1;
                c += dpp<0xB1>(c);
                c += dpp<0x4E>(c);
                // t_k used by every lane here (an empty asm), so its read stays with the step's
                // other reads: the compiler had sunk it into the writer's branch, behind the
                // reduction -- an LDS round trip on every backward step's critical path.  The
                // last level's add folded into the update: (t_k - c) - y, the first
                // subtraction taken while y moves
                asm volatile("" ::"v"(tk));
                double pre = tk - c;
                int jo = j0;
                asm volatile("" : "+v"(pre), "+v"(jo));  // (pre kept out of the branch; the writer test a compare, not a spilled mask)
                const double y = dpp<0x141>(c);
                if (jo == 0) xt[k * S + i] = pre - y;
            }
            __syncthreads();
        }
    }
    SPH(14)
#undef SPH
}

// ---------------------------------------------------------------------------
// The forms measured and not taken (variants 14 / 15, the interface form) live in
// solve_big_exp.h, built into the experimental builds only; k_solve_b names them in branches the
// production instantiations discard.
template <int SL> struct TwoSided4;
template <int SL> struct TwoSidedQ;
template <int NS> struct TwoSidedW;
template <int SL>
__device__ void twisted_solve4(const TwoSided4<SL>& R, const KParams& p, const double* Fc, const double* Gc,
                               const int* toffL, const int (&so)[SL], const int (&fo)[SL], double* rb, double* xt,
                               double* tv, long long* pacc);
template <int SL>
__device__ void iface_solve(const TwoSidedQ<SL>& R, const KParams& p, const double* __restrict__ Fc,
                            const double* __restrict__ Gc, int tvl, double* __restrict__ rb, double* __restrict__ xt,
                            double* __restrict__ tv, double* __restrict__ cor, long long* pacc, long long* pw);
template <int NS>
__device__ void wave_twisted_solve(const TwoSidedW<NS>& R, const KParams& p, const double* Fc, const double* Gc,
                                   const int* toffL, double* rb, double* xt, double* cor, long long* pacc);
#ifdef MPCQP_EXPERIMENTAL
#include "solve_big_exp.h"
#endif

// doubles of the F / G region: F_k rows (k = 1..p), G_k tail rows (k = p..nb-2), and
// at least the four scratch tiles factorize2 needs
template <class KP>
__host__ __device__ inline int big_fg_len(const KP& p) {
    const int fg = (p.pmeet * p.amax + (p.nb - 1 - p.pmeet) * p.bmax) * FGS;
    return fg > 4 * SS ? fg : 4 * SS;
}


// TTK = 512: TwoSided / twisted_solve (nb up to 24); TTK = 128: TwoSidedW / wave_twisted_solve (nb <= 8).
// NS: the most steps one chain takes, max(p, nb-1-p).
template <int TTK, int NS, int K, int CS, int RS, bool IF = false>
__device__ __forceinline__ void solve_b_body(const long b, double* __restrict__ xo, double* __restrict__ yo,
                                             int factor_only) {
    // the lane id and the parameter block (the kernel's first argument, at the start of the
    // kernarg segment) through empty asms per instance: what the body derives from them is
    // formed in the body, not hoisted out of the work loop and held across every solve
    const int tid = opaque_v((int)threadIdx.x);
    KPc* pk = (KPc*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(pk));
    KPc& p = *pk;
#include "solve_big_body.inc"
}

// The kernel: one workgroup per instance in the dispatch order, or -- PERSIST, for a batch
// larger than the resident slots (go_b; MPCQP_PERSIST=0 turns it off) -- one workgroup per
// resident slot taking the next instance of the order from a counter as soon as it finishes one.
// The command processor issues a grid in order and holds it while the next workgroup's XCD has
// no free CU (profiles/r6/dispatch.txt): the persistent form never waits on it.  Its body inlined
// into the loop (solve_b_body, the lane id and the parameter block laundered per instance: 29
// spilled VGPRs without, 40 with the body text in a lambda) keeps one spilled scalar in the
// sweep steps (pinned in tests/test_isa_shape.py) and wins: cfg 5 274.3 k -> 294.2 k.  The
// one-instance form includes the same body text straight into the kernel (solve_big_body.inc),
// so its code is the stand-alone kernel's.  Each instance's arithmetic is the same either way.
template <int TTK, int NS, int K, int CS, int RS, bool IF = false, bool PERSIST = false>
__global__ __launch_bounds__(TTK, 1) void k_solve_b(KParams p, double* __restrict__ xo, double* __restrict__ yo,
                                                   int factor_only) {
    if constexpr (!PERSIST) {
        const int tid = threadIdx.x;
        const long b = instance_of(p);
#include "solve_big_body.inc"
    } else {
    const int tid = threadIdx.x;
    int* const slot = carve(p).L.flag + 8;  // (a flag word the body does not use)
    auto next = [&]() -> long {
        if (tid == 0) *slot = atomicAdd(p.queue, 1);
        __syncthreads();
        const long i = __builtin_amdgcn_readfirstlane(*slot);
        __syncthreads();
        return i;
    };
    long idx = next();
#pragma unroll 1
    while (idx < p.qn) {
        const long b = p.order ? (long)__builtin_amdgcn_readfirstlane(p.order[idx]) : idx;
        solve_b_body<TTK, NS, K, CS, RS, IF>(b, xo, yo, factor_only);
        __syncthreads();
        idx = next();
    }
    if (tid == 0 && atomicAdd(p.queue + 1, 1) == (int)gridDim.x - 1) {
        __hip_atomic_store(p.queue, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(p.queue + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    }
}

size_t lds_solve_bytes_big(const KParams& p) {
    return lds_solve_bytes(p) + 16 + sizeof(double) * (size_t)big_fg_len(p) + sizeof(int) * (size_t)p.nb;
}

#ifdef MPCQP_EXPERIMENTAL
// The interface form: experimental build only, opt-in (MPCQP_BIG_FORM=iface, read once per
// process) -- exact, but slower than the twisted sweep on cfg 5 (38.0 against
// 36.2 ms per launch)
static bool big_iface() {
    static const bool on = [] {
        const char* e = getenv("MPCQP_BIG_FORM");
        return e && !strcmp(e, "iface");
    }();
    return on;
}
#endif

template <int TTK, int NS, int K, int CS, int RS>
static hipError_t go_b(const KParams& p, long B, double* xo, double* yo, int fo, hipStream_t st, KernelRef* ref) {
    const size_t lds = lds_solve_bytes_big(p);
    auto k = k_solve_b<TTK, NS, K, CS, RS>;
#ifdef MPCQP_EXPERIMENTAL
    if constexpr (TTK == 512)
        if (big_iface() && p.ifok) k = k_solve_b<TTK, NS, K, CS, RS, true>;
#endif
    if (ref) { *ref = {(const void*)k, TTK, lds}; return hipSuccess; }
    KParams q = p;
    q.persist = !fo && p.queue && p.qpersist && p.slots > 0 && B > p.slots;
    q.qn = B;
    if (q.persist) {
        k = k_solve_b<TTK, NS, K, CS, RS, false, true>;
#ifdef MPCQP_EXPERIMENTAL
        if constexpr (TTK == 512)
            if (big_iface() && p.ifok) k = k_solve_b<TTK, NS, K, CS, RS, true, true>;
#endif
    }
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3((unsigned)(q.persist ? p.slots : B)), dim3(TTK), lds, st, q, xo, yo, fo);
    return hipGetLastError();
}

hipError_t launch_solve_big(const KParams& p, long B, double* xo, double* yo, int factor_only, hipStream_t st,
                            KernelRef* ref) {
    switch (p.variant) {
        case 11: return go_b<512, 6, 8, 1, 2>(p, B, xo, yo, factor_only, st, ref);   // nb <= 12
        case 12: return go_b<512, 9, 8, 2, 2>(p, B, xo, yo, factor_only, st, ref);   // nb <= 18
        case 13: return go_b<512, 12, 8, 2, 3>(p, B, xo, yo, factor_only, st, ref);  // nb <= 24
#ifdef MPCQP_EXPERIMENTAL
        // 256 threads, one wave per SIMD (twisted_solve4): measured and not taken
        case 15: return go_b<256, 9, 8, 3, 4>(p, B, xo, yo, factor_only, st, ref);   // nb <= 18
        case 14: return go_b<128, 4, 8, 2, 2>(p, B, xo, yo, factor_only, st, ref);   // nb <= 8, two waves
#endif
        default: return hipErrorInvalidValue;
    }
}

}  // namespace mpcqp
