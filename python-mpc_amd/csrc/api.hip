// api.hip -- C ABI of libmpcqp.so (declared in include/mpcqp.h).
//
// Host side of the drop-in boundary for `osqp.OSQP().setup()/update()/solve()`
// (vehicle_lateral_mpc_slack_increment.py:118-121,237,248,269;
// Control/MPC/mpc_dynamics.py:392-396).  The host only performs the symbolic
// analysis of the shared sparsity pattern (plan.cpp), memory management and
// kernel launches; every per-instance number is computed by the HIP kernels in
// kernels.hip.  There is no CPU fallback: without a HIP device every entry
// point that needs one returns MPCQP_EDEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/mpcqp.h"
#include "kernels.h"
#include "plan.h"

using namespace mpcqp;

namespace {

thread_local std::string g_err;

// MPCQP_SETUP_TRACE=1 (diagnostic): the host-side stages of a setup call, in microseconds
// since the previous mark, on stderr
struct SetupTrace {
    bool on = false;
    std::chrono::steady_clock::time_point t;
    SetupTrace() {
        const char* e = getenv("MPCQP_SETUP_TRACE");
        on = e && e[0] == '1';
        t = std::chrono::steady_clock::now();
    }
    void mark(const char* what) {
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "mpcqp setup: %-22s %8.1f us\n", what,
                std::chrono::duration<double, std::micro>(now - t).count());
        t = now;
    }
};
SetupTrace& strace() {
    static thread_local SetupTrace tr;
    return tr;
}

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

}  // namespace

// shared with the other translation units of the library (mpc_device.hip)
int mpcqp::set_error(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

namespace {

#define HIPCHK(expr)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return fail(MPCQP_EDEVICE, "%s failed: %s", #expr, hipGetErrorString(e_));      \
    } while (0)

struct Shard {
    int dev = 0;
    long b0 = 0, B = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // stream ordering of the calls on the handle: last_st is the stream of the last
    // call; a call on another stream records last_ev there and waits for it (enter)
    hipEvent_t last_ev = nullptr;
    hipStream_t last_st = nullptr;
    int* dplan = nullptr;
    void* dws = nullptr;    // one allocation for the whole workspace
    void* dio = nullptr;    // staging for the host-pointer API
    double *in_Px = nullptr, *in_Ax = nullptr, *in_q = nullptr, *in_l = nullptr, *in_u = nullptr;
    double *out_x = nullptr, *out_y = nullptr;
    // host-pointer API, small shards: pinned staging of everything a solve returns (x, y, the
    // info, the certificates, the statuses), filled by mpcqp_solve_batch with one
    // synchronisation; the info / certificate / polish getters then read it (mpcqp_handle::staged)
    char* hstage = nullptr;
    char* dstage = nullptr;  // the device side of hstage (launch_gather)
    char* hin = nullptr;  // ... and of update()'s q, l, u and the error flags it reads back
    size_t dws_bytes = 0, dplan_bytes = 0, hstage_bytes = 0, hin_bytes = 0, dstage_bytes = 0;  // (resource pool keys)
    unsigned long long dplan_tag = 0;  // Plan::uid of the device plan copy
    KParams kp{};
};

}  // namespace

struct mpcqp_handle {
    std::shared_ptr<const Plan> plan;  // shared with the plan cache (read-only)
    std::vector<int32_t> Pp, Pi, Ap, Ai;  // the user's pattern (a re-plan: replan_plain)
    mpcqp_settings set{};
    int n = 0, m = 0;
    long B = 0;
    std::vector<Shard> shards;
    bool timed = false;
    double last_ms = -1.0;
    bool collect = false;        // record hipEvent pairs around device solve launches
    bool collect_setup = false;  // ... and around device setup launches
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_setup, ev_solve;
    std::pair<hipEvent_t, hipEvent_t> last_pair{nullptr, nullptr};  // events of the last device solve
    bool staged = false;  // every shard's hstage holds the last mpcqp_solve_batch's results
    bool one_shot = false;    // mpcqp_set_one_shot: setup_solve_device persists no workspace state
    bool state_gone = false;  // the last setup was one-shot: calls that read the workspace refuse
};

namespace {

// calls that read what a setup leaves in the workspace (the scaled data, the iterates, the
// certificates) after a one-shot setup + solve, which left none of it
int need_state(const mpcqp_handle* h, const char* what) {
    if (h && h->state_gone)
        return fail(MPCQP_EINVAL, "%s: the last setup was one-shot (mpcqp_set_one_shot): the workspace keeps no "
                    "state; call a setup first", what);
    return 0;
}

template <class T>
size_t carve(size_t& off, size_t count) {
    off = (off + 255) & ~(size_t)255;
    size_t o = off;
    off += count * sizeof(T);
    return o;
}

// the plan-shape fields of KParams (what variant_fits reads)
void shape_params(const Plan& pl, KParams& k) {
    k.n = pl.n; k.m = pl.m; k.nb = pl.nb; k.npad = pl.npad; k.nnzP = pl.nnzP; k.nnzA = pl.nnzA; k.amax = pl.amax;
    k.bmax = pl.bmax; k.pmeet = (pl.nb - 1) / 2;
    k.ifok = pl.nb > 4 && pl.nb <= 64 && pl.amax <= 16 && pl.bmax <= 16 && pl.toff[k.pmeet] >= pl.amax &&
             pl.toff[k.pmeet] + pl.bmax <= kS;
    k.bsz01 = k.bsz23 = 1 << 20;
    if (pl.nb == 4) {
        k.bsz01 = std::max(pl.bsize[0], pl.bsize[1]);
        k.bsz23 = std::max(pl.bsize[2], pl.bsize[3]);
    }
    k.gk = pl.gather_k; k.pk = pl.p_k; k.ntgt = pl.ntgt; k.term_max = pl.term_max;
    k.gk1 = 0;
    for (int i = 128; i < pl.m; ++i) k.gk1 = std::max(k.gk1, pl.acsr_ptr[i + 1] - pl.acsr_ptr[i]);
    k.ne = pl.ne; k.ecnt = pl.ecnt; k.eterm_max = pl.eterm_max;
    k.gkr = pl.max_row_nnz; k.gkc = pl.max_col_nnz;
}

// ---- resource pool ----
// Device blocks, pinned host blocks and streams (with their three events) of freed handles,
// kept for the next handle of the same shape: the Control/MPC scripts set up a fresh osqp
// object every control step, and creating / destroying these costs most of a small setup
// (~0.4 ms).  A reused block is cleared exactly as a new one (alloc_shard's memset), a reused
// stream is idle (mpcqp_free synchronises it first).  Bounded: 256 MiB of device blocks,
// 64 MiB pinned, 8 streams; past that, resources are released as before.  The pool is never
// torn down (process exit reclaims it; no HIP call runs from a static destructor).
struct ResPool {
    struct Blk { int dev; size_t bytes; void* p; unsigned long long tag; };
    struct Str { int dev; hipStream_t st; hipEvent_t e0, e1, el; };
    std::mutex mu;
    std::vector<Blk> dev, pin;
    std::vector<Str> str;
    size_t dev_total = 0, pin_total = 0;
};
ResPool& respool() {
    static ResPool* p = new ResPool;
    return *p;
}
constexpr size_t kPoolDev = 256u << 20, kPoolPin = 64u << 20;
constexpr size_t kPoolStreams = 8;

// tag: what a block holds (a device plan's Plan::uid; 0 nothing reusable).  A block with the
// asked-for tag is preferred, and *hit says whether it was found (its contents are then the
// same as the caller would write).
hipError_t pool_malloc(int dev, size_t bytes, void** out, bool pinned, unsigned long long tag = 0,
                       bool* hit = nullptr) {
    ResPool& r = respool();
    if (hit) *hit = false;
    {
        std::lock_guard<std::mutex> lk(r.mu);
        auto& v = pinned ? r.pin : r.dev;
        size_t pick = v.size();
        for (size_t i = v.size(); i-- > 0;)
            if (v[i].dev == dev && v[i].bytes == bytes) {
                if (tag && v[i].tag == tag) { pick = i; break; }
                if (pick == v.size()) pick = i;
            }
        if (pick < v.size()) {
            *out = v[pick].p;
            if (hit) *hit = tag && v[pick].tag == tag;
            (pinned ? r.pin_total : r.dev_total) -= bytes;
            v.erase(v.begin() + pick);
            return hipSuccess;
        }
    }
    hipError_t e = pinned ? hipHostMalloc(out, bytes, hipHostMallocDefault) : hipMalloc(out, bytes);
    if (e == hipSuccess) return e;
    // out of memory: give the pooled blocks of this kind back (a caller that freed a handle to
    // make room must not fail where hipFree would have returned the memory) and try once more
    (void)hipGetLastError();
    std::vector<ResPool::Blk> rel;
    {
        std::lock_guard<std::mutex> lk(r.mu);
        auto& v = pinned ? r.pin : r.dev;
        for (size_t i = v.size(); i-- > 0;)
            if (pinned || v[i].dev == dev) {
                rel.push_back(v[i]);
                (pinned ? r.pin_total : r.dev_total) -= v[i].bytes;
                v.erase(v.begin() + i);
            }
    }
    if (rel.empty()) return e;
    for (auto& b : rel) {
        if (pinned) (void)hipHostFree(b.p);
        else (void)hipFree(b.p);
    }
    return pinned ? hipHostMalloc(out, bytes, hipHostMallocDefault) : hipMalloc(out, bytes);
}
void pool_free(int dev, size_t bytes, void* p, bool pinned, unsigned long long tag = 0) {
    if (!p) return;
    ResPool& r = respool();
    {
        std::lock_guard<std::mutex> lk(r.mu);
        size_t& tot = pinned ? r.pin_total : r.dev_total;
        if (tot + bytes <= (pinned ? kPoolPin : kPoolDev)) {
            (pinned ? r.pin : r.dev).push_back({dev, bytes, p, tag});
            tot += bytes;
            return;
        }
    }
    if (pinned) (void)hipHostFree(p);
    else (void)hipFree(p);
}
int pool_stream(Shard& s) {
    ResPool& r = respool();
    {
        std::lock_guard<std::mutex> lk(r.mu);
        for (size_t i = r.str.size(); i-- > 0;)
            if (r.str[i].dev == s.dev) {
                s.stream = r.str[i].st; s.ev0 = r.str[i].e0; s.ev1 = r.str[i].e1; s.last_ev = r.str[i].el;
                r.str.erase(r.str.begin() + i);
                return 0;
            }
    }
    HIPCHK(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
    HIPCHK(hipEventCreate(&s.ev0));
    HIPCHK(hipEventCreate(&s.ev1));
    HIPCHK(hipEventCreateWithFlags(&s.last_ev, hipEventDisableTiming));
    return 0;
}
void pool_stream_release(Shard& s) {
    if (!s.stream) return;
    ResPool& r = respool();
    {
        std::lock_guard<std::mutex> lk(r.mu);
        if (r.str.size() < kPoolStreams && s.ev0 && s.ev1 && s.last_ev) {
            r.str.push_back({s.dev, s.stream, s.ev0, s.ev1, s.last_ev});
            return;
        }
    }
    if (s.ev0) (void)hipEventDestroy(s.ev0);
    if (s.ev1) (void)hipEventDestroy(s.ev1);
    if (s.last_ev) (void)hipEventDestroy(s.last_ev);
    (void)hipStreamDestroy(s.stream);
}

int upload_plan(const Plan& pl, Shard& s) {
    std::vector<const std::vector<int>*> parts = {
        &pl.pad_var, &pl.acsc_ptr, &pl.acsc_row, &pl.acsc_v, &pl.acsr_ptr, &pl.acsr_col, &pl.acsr_v,
        &pl.psym_ptr, &pl.psym_col, &pl.psym_v, &pl.p_r, &pl.p_c, &pl.a_r, &pl.a_c,
        &pl.asm_blk_ptr, &pl.asm_tgt, &pl.tterm, &pl.acsr_pos, &pl.gcol, &pl.grow, &pl.gpsym, &pl.toff, &pl.bsize, &pl.tcnt,
        &pl.eown, &pl.etterm, &pl.wide_cg, &pl.wide_pg, &pl.wide_rg, &pl.wide_as, &pl.wide_ps, &pl.csc_pos};
    std::vector<size_t> offs;
    size_t total = 0;
    for (auto* v : parts) {
        offs.push_back(total);
        total += v->size() + 1;  // never allocate zero-length parts
    }
    s.dplan_bytes = total * sizeof(int);
    s.dplan_tag = pl.uid;
    bool have = false;  // a pooled copy of this very plan (a fresh handle of the same pattern)
    HIPCHK(pool_malloc(s.dev, s.dplan_bytes, (void**)&s.dplan, false, pl.uid, &have));
    if (!have) {  // (the flat image is built only when it is uploaded)
        std::vector<int> flat;
        flat.reserve(total);
        for (auto* v : parts) {
            flat.insert(flat.end(), v->begin(), v->end());
            flat.push_back(0);
        }
        HIPCHK(hipMemcpy(s.dplan, flat.data(), flat.size() * sizeof(int), hipMemcpyHostToDevice));
    }
    const int** dst[] = {&s.kp.pad_var, &s.kp.acsc_ptr, &s.kp.acsc_row, &s.kp.acsc_v, &s.kp.acsr_ptr,
                         &s.kp.acsr_col, &s.kp.acsr_v, &s.kp.psym_ptr, &s.kp.psym_col, &s.kp.psym_v,
                         &s.kp.p_r, &s.kp.p_c, &s.kp.a_r, &s.kp.a_c, &s.kp.asm_blk_ptr, &s.kp.asm_tgt,
                         &s.kp.tterm, &s.kp.acsr_pos,
                         &s.kp.gcol, &s.kp.grow, &s.kp.gpsym, &s.kp.toff, &s.kp.bsize, &s.kp.tcnt,
                         &s.kp.eown, &s.kp.etterm, &s.kp.wcg, &s.kp.wpg, &s.kp.wrg, &s.kp.was, &s.kp.wps,
                         &s.kp.csc_pos};
    for (size_t i = 0; i < parts.size(); ++i) *dst[i] = s.dplan + offs[i];
    return 0;
}

size_t workspace_bytes(const Plan& pl, long B, bool with_io) {
    size_t off = 0;
    const long n = pl.n, m = pl.m, np = pl.npad, nb = pl.nb;
    const long SS = (long)kS * kS;
    carve<double>(off, B * pl.nnzP); carve<double>(off, B * pl.nnzA);
    carve<double>(off, B * np); carve<double>(off, B * np);            // q, D
    carve<double>(off, B * m); carve<double>(off, B * m); carve<double>(off, B * m);  // l u E
    carve<double>(off, B * np); carve<double>(off, B * m); carve<double>(off, B * m); // x z y
    carve<double>(off, B * 4);
    carve<double>(off, B * nb * SS); carve<double>(off, B * nb * SS); carve<double>(off, B * nb * SS);
    carve<double>(off, B * dense_rows_doubles(pl.nb, pl.ne));       // Kd
    carve<double>(off, B * m); carve<double>(off, B * n);              // certificates
    for (int i = 0; i < 4; ++i) carve<double>(off, B);
    carve<signed char>(off, B * m);
    for (int i = 0; i < 8; ++i) carve<int>(off, B);
    carve<int>(off, 1);  // done (fused order epilogue)
    carve<int>(off, 2);  // queue (k_solve_b's persistent form)
    carve<long long>(off, B * kProfSlots);
    carve<KParams>(off, 1);
    if (with_io) {
        carve<double>(off, B * pl.nnzP); carve<double>(off, B * pl.nnzA);
        carve<double>(off, B * n); carve<double>(off, B * m); carve<double>(off, B * m);
        carve<double>(off, B * n); carve<double>(off, B * m);
    }
    return off + 256;
}

// sync: wait for the zeroing, the identity order and the parameter block before returning (the
// device API's callers may use the workspace from any stream; the host batch setup queues all
// its work on the shard's stream behind them and waits once, in check_setup)
int alloc_shard(mpcqp_handle* h, Shard& s, bool with_io, bool sync = true) {
    const Plan& pl = *h->plan;
    HIPCHK(hipSetDevice(s.dev));
    if (int e = pool_stream(s)) return e;
    strace().mark("stream");
    if (int e = upload_plan(pl, s)) return e;
    strace().mark("plan upload");
    const long B = s.B, n = pl.n, m = pl.m, np = pl.npad, nb = pl.nb;
    const long SS = (long)kS * kS;
    size_t total = workspace_bytes(pl, B, with_io);
    hipError_t e = pool_malloc(s.dev, total, &s.dws, false);
    if (e == hipSuccess) s.dws_bytes = total;
    if (e != hipSuccess)
        return fail(MPCQP_ENOMEM, "hipMalloc(%zu bytes) failed: %s", total, hipGetErrorString(e));
    strace().mark("workspace alloc");
    HIPCHK(hipMemsetAsync(s.dws, 0, total, s.stream));
    strace().mark("workspace memset");
    char* base = (char*)s.dws;
    size_t off = 0;
    KParams& k = s.kp;
    k.Px = (double*)(base + carve<double>(off, B * pl.nnzP));
    k.Ax = (double*)(base + carve<double>(off, B * pl.nnzA));
    k.q = (double*)(base + carve<double>(off, B * np));
    k.D = (double*)(base + carve<double>(off, B * np));
    k.l = (double*)(base + carve<double>(off, B * m));
    k.u = (double*)(base + carve<double>(off, B * m));
    k.E = (double*)(base + carve<double>(off, B * m));
    k.x = (double*)(base + carve<double>(off, B * np));
    k.z = (double*)(base + carve<double>(off, B * m));
    k.y = (double*)(base + carve<double>(off, B * m));
    k.scal = (double*)(base + carve<double>(off, B * 4));
    k.F = (double*)(base + carve<double>(off, B * nb * SS));
    k.H = (double*)(base + carve<double>(off, B * nb * SS));
    k.Si = (double*)(base + carve<double>(off, B * nb * SS));
    k.Kd = dense_rows_doubles(pl.nb, pl.ne) ? (double*)(base + carve<double>(off, B * dense_rows_doubles(pl.nb, pl.ne)))
                                            : nullptr;
    k.dyc = (double*)(base + carve<double>(off, B * m));
    k.dxc = (double*)(base + carve<double>(off, B * n));
    k.obj = (double*)(base + carve<double>(off, B));
    k.pri = (double*)(base + carve<double>(off, B));
    k.dua = (double*)(base + carve<double>(off, B));
    k.rho_est = (double*)(base + carve<double>(off, B));
    k.ct = (signed char*)(base + carve<signed char>(off, B * m));
    k.err = (int*)(base + carve<int>(off, B));  // (err right before status: check_setup reads both in one copy)
    k.status = (int*)(base + carve<int>(off, B));
    k.iter = (int*)(base + carve<int>(off, B));
    k.rho_upd = (int*)(base + carve<int>(off, B));
    k.pstat = (int*)(base + carve<int>(off, B));
    k.ffresh = (int*)(base + carve<int>(off, B));  // zero from the memset above
    k.reuse = !(getenv("MPCQP_FACTOR_REUSE") && getenv("MPCQP_FACTOR_REUSE")[0] == '0');
    k.apart = !(getenv("MPCQP_MIDDLE_APART") && getenv("MPCQP_MIDDLE_APART")[0] == '0');
    k.lchain = !(getenv("MPCQP_LDS_CHAIN") && getenv("MPCQP_LDS_CHAIN")[0] == '0');
    {  // dispatch order (kernels.hip::k_order), identity until the first solve
        int* ord = (int*)(base + carve<int>(off, B));
        HIPCHK(launch_iota(ord, B, s.stream));
        k.order = ord;
        k.pred = (int*)(base + carve<int>(off, B));  // zero from the memset above
        const char* od = getenv("MPCQP_ORDER_DECAY");
        k.odecay = od ? std::max(0, std::min(8, atoi(od))) : 7;  // (tools/pred_sim.py, profiles/r6/dispatch.txt)
        strace().mark("order upload");
        if (const char* ev = getenv("MPCQP_DISPATCH"); ev && !strcmp(ev, "identity")) k.order = nullptr;  // A/B
    }
    int* const done = (int*)(base + carve<int>(off, 1));  // zero from the memset above
    k.queue = (int*)(base + carve<int>(off, 2));          // zero from the memset above
    k.qpersist = !(getenv("MPCQP_PERSIST") && getenv("MPCQP_PERSIST")[0] == '0');
    k.persist = 0;
    k.qn = 0;
    k.prof = nullptr;
    if (const char* ev = getenv("MPCQP_PHASE_PROF"); ev && ev[0] == '1')
        k.prof = (long long*)(base + carve<long long>(off, B * kProfSlots));
    if (with_io) {
        s.in_Px = (double*)(base + carve<double>(off, B * pl.nnzP));
        s.in_Ax = (double*)(base + carve<double>(off, B * pl.nnzA));
        s.in_q = (double*)(base + carve<double>(off, B * n));
        s.in_l = (double*)(base + carve<double>(off, B * m));
        s.in_u = (double*)(base + carve<double>(off, B * m));
        s.out_x = (double*)(base + carve<double>(off, B * n));
        s.out_y = (double*)(base + carve<double>(off, B * m));
    }
    shape_params(pl, k);
    const mpcqp_settings& st = h->set;
    k.sigma = st.sigma; k.alpha = st.alpha; k.eps_abs = st.eps_abs; k.eps_rel = st.eps_rel;
    k.eps_pinf = st.eps_prim_inf; k.eps_dinf = st.eps_dual_inf; k.rho0 = st.rho;
    k.rho_tol = st.adaptive_rho_tolerance;
    k.max_iter = st.max_iter; k.scaling = st.scaling; k.check_term = st.check_termination;
    k.warm_start = st.warm_start; k.adaptive_rho = st.adaptive_rho; k.scaled_term = st.scaled_termination;
    k.polish = st.polish; k.refine_iter = st.polish_refine_iter; k.delta = st.delta;
    int interval = st.adaptive_rho_interval;
    if (st.adaptive_rho && interval == 0) interval = st.check_termination ? 4 * st.check_termination : 100;
    k.rho_interval = interval;
    if (solve_variant(k) < 0)
        return fail(MPCQP_EUNSUPPORTED, "problem shape outside the solve kernel's instantiations (n=%d m=%d)", pl.n, pl.m);
    k.variant = solve_variant(k);
    if (const char* ev = getenv("MPCQP_VARIANT"); ev && *ev) {  // diagnostic override (A/B timing)
        const int v = atoi(ev);
        if (!variant_fits(k, v)) return fail(MPCQP_EUNSUPPORTED, "MPCQP_VARIANT=%d does not fit this plan", v);
        k.variant = v;
    }
    k.mode = solve_mode(k.variant);
    // k_solve_w2 sorts the next dispatch order in its last workgroup (MPCQP_ORDER_KERNEL=1: k_order)
    k.done = nullptr;
    if ((k.variant == 10 || k.variant == 17 || k.variant == 19) && k.order &&
        !(getenv("MPCQP_ORDER_KERNEL") && getenv("MPCQP_ORDER_KERNEL")[0] == '1'))
        k.done = done;
    {  // resident solve workgroups: below this batch size the dispatch order is moot
        int ncu = 0;
        HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, s.dev));
        const int occ = solve_blocks_per_cu(k);
        if (occ < 0) return fail(MPCQP_EDEVICE, "occupancy query for solve variant %d failed", k.variant);
        k.slots = (long)ncu * occ;
    }
    strace().mark("variant + occupancy");
    k.self = (const KParams*)(base + carve<KParams>(off, 1));
    // the zeroing, the identity order and the parameter block in stream order, one wait for
    // all three (callers then use the workspace from any stream or from the host)
    HIPCHK(hipMemcpyAsync((void*)k.self, &k, sizeof(KParams), hipMemcpyHostToDevice, s.stream));
    if (sync) HIPCHK(hipStreamSynchronize(s.stream));
    strace().mark("params upload");
    if (size_t lds = lds_kernel_bytes(k); lds > 160 * 1024)
        return fail(MPCQP_EUNSUPPORTED, "problem needs %zu bytes of LDS per instance (> 160 KiB)", lds);
    return 0;
}

// The plan of a handle: with the degree <= 1 vertices of K eliminated (plan.h) when the
// four-wave kernel then runs the reduced system -- the slack layouts (SURVEY.md §8
// configs 1, 3, 4: 230 variables, 8 blocks -> 125 in 4) -- else the plain plan.  Polish
// factors the full system (factorize<POL>), so it keeps the plain plan; MPCQP_ELIM=0 (A/B)
// and an MPCQP_VARIANT override other than 17 do too.
// The plan's choice and, when an eliminated plan is rejected, why (Plan::choice /
// choice_note; MPCQP_PLAN_LOG=1 prints it): a regression in the level ordering or the
// greedy packing (e.g. amax > 8) then shows up in plan_info instead of as a quiet 2x
// slowdown on the plain plan.
std::string w4_misfit(const KParams& k) {
    char buf[256];
    const bool el = k.ne > 0;
    std::string r;
    auto need = [&](bool ok, const char* what, long have, long lim) {
        if (ok) return;
        snprintf(buf, sizeof buf, "%s%s = %ld > %ld", r.empty() ? "" : ", ", what, have, lim);
        r += buf;
    };
    if (k.nb != 4) {
        snprintf(buf, sizeof buf, "nb = %d (needs 4)", k.nb);
        r += buf;
    }
    need(k.amax <= 8, "amax", k.amax, 8);
    need(k.gkr <= 6, "longest A row", k.gkr, 6);
    need(k.gkc <= (el ? 8 : 6), "longest A column", k.gkc, el ? 8 : 6);
    need(k.pk <= 4, "longest P column", k.pk, 4);
    need(k.m <= 256, "m", k.m, 256);
    need(k.npad <= (el ? 256 : 128), "npad", k.npad, el ? 256 : 128);
    need(k.nnzA <= (el ? 768 : 512), "nnzA", k.nnzA, el ? 768 : 512);
    need(k.nnzP <= 256, "nnzP", k.nnzP, 256);
    if (el) need(k.ecnt <= 2, "A nonzeros of an eliminated column", k.ecnt, 2);
    if (el) need(k.ne <= 128, "eliminated columns", k.ne, 128);
    KParams q2 = k;
    q2.mode = 2;
    need(lds_w2_bytes(q2) <= 80 * 1024, "LDS bytes", (long)lds_w2_bytes(q2), 80 * 1024);
    return r.empty() ? "does not fit variant 17" : r;
}

unsigned long long next_plan_uid() {
    static std::atomic<unsigned long long> c{0};
    return ++c;
}

std::string choose_plan(int32_t n, int32_t m, const int32_t* Pp, const int32_t* Pi, const int32_t* Ap,
                        const int32_t* Ai, const mpcqp_settings& st, Plan& pl) {
    const char* ev = getenv("MPCQP_ELIM");
    const char* vv = getenv("MPCQP_VARIANT");
    int choice = 0;
    std::string note;
    if (!st.polish && !(ev && ev[0] == '0') && !(vv && *vv && atoi(vv) != 17)) {
        std::string err = build_plan(n, m, Pp, Pi, Ap, Ai, pl, true);
        if (err.empty() && pl.ne > 0) {  // (nothing eliminated: the plain plan, level-merged blocks)
            KParams k{};
            shape_params(pl, k);
            k.mode = 2;
            if (variant_fits(k, 17)) {
                pl.choice = 1;
                pl.uid = next_plan_uid();
                return err;
            }
            choice = 2;
            note = "eliminated plan (" + std::to_string(pl.ne) + " columns, " + std::to_string(pl.nb) +
                   " blocks) rejected: " + w4_misfit(k);
        } else {
            choice = err.empty() ? 3 : 2;
            if (!err.empty()) note = "eliminated plan failed: " + err;
        }
    }
    std::string err = build_plan(n, m, Pp, Pi, Ap, Ai, pl, false, true);  // (balanced four-block merge: plan.cpp)
    pl.uid = next_plan_uid();
    pl.choice = choice;
    pl.choice_note = note;
    if (const char* lg = getenv("MPCQP_PLAN_LOG"); lg && lg[0] == '1' && !note.empty())
        fprintf(stderr, "mpcqp: %s; using the plain plan\n", note.c_str());
    return err;
}

// Plans by sparsity pattern: the Control/MPC scripts set up a fresh osqp object, with the same
// pattern, every control step (mpc_kinematics.py:194-198), and planning is most of a small
// setup's host time (~0.8 ms at N = 20).  A few recent plans are kept; a hit compares the whole
// pattern, the polish flag and the plan-choice overrides, so it returns exactly the plan
// choose_plan would build.
struct PlanKey {
    int32_t n = 0, m = 0;
    bool polish = false;
    std::string env;
    std::vector<int32_t> pat;
    bool operator==(const PlanKey& o) const {
        return n == o.n && m == o.m && polish == o.polish && env == o.env && pat == o.pat;
    }
};
std::mutex g_plan_mu;
std::vector<std::pair<PlanKey, std::shared_ptr<const Plan>>> g_plans;  // most recently used last
constexpr size_t kPlanCache = 8;

std::string cached_plan(int32_t n, int32_t m, const int32_t* Pp, const int32_t* Pi, const int32_t* Ap,
                        const int32_t* Ai, const mpcqp_settings& st, std::shared_ptr<const Plan>& out) {
    auto fresh = [&]() {
        auto pl = std::make_shared<Plan>();
        std::string err = choose_plan(n, m, Pp, Pi, Ap, Ai, st, *pl);
        out = pl;
        return err;
    };
    if (n <= 0 || m < 0 || Pp[n] < 0 || Ap[n] < 0) return fresh();
    PlanKey k;
    k.n = n;
    k.m = m;
    k.polish = st.polish != 0;
    const char* ev = getenv("MPCQP_ELIM");
    const char* vv = getenv("MPCQP_VARIANT");
    k.env = std::string(ev ? ev : "") + "|" + (vv ? vv : "");
    k.pat.reserve(2 * ((size_t)n + 1) + (size_t)Pp[n] + (size_t)Ap[n]);
    k.pat.insert(k.pat.end(), Pp, Pp + n + 1);
    k.pat.insert(k.pat.end(), Pi, Pi + Pp[n]);
    k.pat.insert(k.pat.end(), Ap, Ap + n + 1);
    k.pat.insert(k.pat.end(), Ai, Ai + Ap[n]);
    {
        std::lock_guard<std::mutex> lk(g_plan_mu);
        for (size_t i = g_plans.size(); i-- > 0;)
            if (g_plans[i].first == k) {
                out = g_plans[i].second;  // shared, not copied (a cfg-5 plan copy took ~35 us)
                std::rotate(g_plans.begin() + i, g_plans.begin() + i + 1, g_plans.end());
                return std::string();
            }
    }
    std::string err = fresh();
    if (err.empty()) {
        std::lock_guard<std::mutex> lk(g_plan_mu);
        g_plans.emplace_back(std::move(k), out);
        if (g_plans.size() > kPlanCache) g_plans.erase(g_plans.begin());
    }
    return err;
}

int validate_settings(const mpcqp_settings& s) {
    if (!(s.rho > 0) || !(s.sigma > 0) || s.max_iter <= 0 || s.eps_abs < 0 || s.eps_rel < 0 ||
        (s.eps_abs == 0 && s.eps_rel == 0) || !(s.eps_prim_inf > 0) || !(s.eps_dual_inf > 0) ||
        !(s.alpha > 0 && s.alpha < 2) || s.scaling < 0 || s.check_termination < 0 ||
        s.adaptive_rho_interval < 0 || !(s.adaptive_rho_tolerance >= 1))
        return fail(MPCQP_EINVAL, "invalid settings");
    if (s.polish && (!(s.delta > 0) || s.polish_refine_iter < 0)) return fail(MPCQP_EINVAL, "invalid polish settings");
    return 0;
}

int make_handle(int32_t n, int32_t m, const int32_t* Pp, const int32_t* Pi, const int32_t* Ap,
                const int32_t* Ai, int64_t B, const mpcqp_settings* settings, std::vector<int> devs,
                bool with_io, mpcqp_handle** out) {
    if (!out) return fail(MPCQP_EINVAL, "out is NULL");
    *out = nullptr;
    if (B <= 0) return fail(MPCQP_EINVAL, "batch must be positive");
    if (!Pp || !Pi || !Ap || !Ai) return fail(MPCQP_EINVAL, "NULL pattern array");
    auto h = std::make_unique<mpcqp_handle>();
    if (settings) h->set = *settings;
    else mpcqp_default_settings(&h->set);
    if (int e = validate_settings(h->set)) return e;
    strace().mark("(enter)");
    std::string err = cached_plan(n, m, Pp, Pi, Ap, Ai, h->set, h->plan);
    strace().mark("plan");
    if (!err.empty()) {
        bool unsup = err.rfind("unsupported", 0) == 0;
        return fail(unsup ? MPCQP_EUNSUPPORTED : MPCQP_EINVAL, "%s", err.c_str());
    }
    h->n = n; h->m = m; h->B = B;
    h->Pp.assign(Pp, Pp + n + 1); h->Pi.assign(Pi, Pi + Pp[n]);
    h->Ap.assign(Ap, Ap + n + 1); h->Ai.assign(Ai, Ai + Ap[n]);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(MPCQP_EDEVICE, "no HIP device available (the solver has no CPU fallback)");
    for (int d : devs)
        if (d < 0 || d >= ndev) return fail(MPCQP_EDEVICE, "device %d not present (%d devices)", d, ndev);
    const long nd = (long)devs.size();
    for (long i = 0; i < nd; ++i) {
        Shard s;
        s.dev = devs[i];  // devs may repeat a device (MPCQP_SPLIT): several shards on it, one stream each
        s.b0 = B * i / nd;
        s.B = B * (i + 1) / nd - s.b0;
        if (s.B <= 0) continue;
        h->shards.push_back(s);
    }
    for (auto& s : h->shards)
        if (int e = alloc_shard(h.get(), s, with_io, !with_io)) { mpcqp_free(h.release()); return e; }
    *out = h.release();
    return 0;
}

int check_bounds_host(const mpcqp_handle* h, const double* l, const double* u, long B) {
    if (!l || !u) return 0;
    const long m = h->m;
    for (long i = 0; i < B * m; ++i) {
        double li = std::max(l[i], -1e30), ui = std::min(u[i], 1e30);
        if (!(li <= ui))
            return fail(MPCQP_EINVAL, "instance %ld row %ld: lower bound must be lower than or equal to upper bound",
                        i / m, i % m);
    }
    return 0;
}

// waits for the handle's own streams and for the last call's work wherever it was
// enqueued (a caller stream of the *_device entry points: last_ev)
int sync_all(mpcqp_handle* h) {
    for (auto& s : h->shards) {
        HIPCHK(hipSetDevice(s.dev));
        HIPCHK(hipStreamSynchronize(s.stream));
        if (s.last_st) HIPCHK(hipEventSynchronize(s.last_ev));
    }
    return 0;
}

// Every call enqueues on one stream; work of the previous call on the handle that went
// to another stream is waited for first.  The handle's workspace -- including the
// dispatch order each solve rewrites for the next (kernels.hip::k_order) -- is then
// never read by one stream while another writes it, whatever streams the caller uses.
// stream_leave records last_ev on a caller's stream once the call's work is enqueued, so
// stream_enter never touches a stream of an earlier call (which the caller may have
// destroyed since): on a change of stream it only makes the new stream wait for last_ev.
// The handle's own stream is never destroyed before the handle, so a call on it records
// nothing: last_ev is recorded there only when the next call moves to another stream
// (a single-stream caller's queue holds kernels only -- no event packet between them).
int stream_enter(Shard& s, hipStream_t st) {
    if (s.last_st && s.last_st != st) {
        if (s.last_st == s.stream) HIPCHK(hipEventRecord(s.last_ev, s.stream));
        HIPCHK(hipStreamWaitEvent(st, s.last_ev, 0));
    }
    return 0;
}
int stream_leave(Shard& s, hipStream_t st) {
    if (st != s.stream) HIPCHK(hipEventRecord(s.last_ev, st));
    s.last_st = st;
    return 0;
}

int check_err_flags(mpcqp_handle* h) {
    for (auto& s : h->shards) {
        std::vector<int> err(s.B);
        HIPCHK(hipSetDevice(s.dev));
        HIPCHK(hipMemcpy(err.data(), s.kp.err, sizeof(int) * s.B, hipMemcpyDeviceToHost));
        for (long i = 0; i < s.B; ++i)
            if (err[i]) return fail(MPCQP_EINVAL, "instance %ld: invalid data (l > u or NaN bounds)", s.b0 + i);
    }
    return 0;
}

// The staging layout of one shard (Bs instances): x (Bs n), y (Bs m), obj, pri, dua, rho_est
// (Bs each), the certificates dxc (Bs n) and dyc (Bs m) as doubles, then status, iter,
// rho_upd, pstat (Bs each) as ints.  Shards past kStageMax bytes copy straight into the
// caller's buffers as before (the large throughput batches, where the copies dominate).
constexpr size_t kStageMax = 16u << 20;
size_t stage_bytes(const mpcqp_handle* h, long Bs) {
    return sizeof(double) * (size_t)Bs * (2 * (size_t)h->n + 2 * (size_t)h->m + 4) + sizeof(int) * 4 * (size_t)Bs;
}
struct Stage {
    double *x, *y, *obj, *pri, *dua, *rho_est, *dxc, *dyc;
    int *status, *iter, *rho_upd, *pstat;
};
Stage stage_of(const mpcqp_handle* h, const Shard& s) {
    Stage g;
    double* d = (double*)s.hstage;
    const long Bs = s.B, n = h->n, m = h->m;
    g.x = d; g.y = g.x + Bs * n; g.obj = g.y + Bs * m; g.pri = g.obj + Bs; g.dua = g.pri + Bs;
    g.rho_est = g.dua + Bs; g.dxc = g.rho_est + Bs; g.dyc = g.dxc + Bs * n;
    int* q = (int*)(g.dyc + Bs * m);
    g.status = q; g.iter = q + Bs; g.rho_upd = q + 2 * Bs; g.pstat = q + 3 * Bs;
    return g;
}

// osqp_setup's convexity test (OSQP 0.6 init_linsys_solver: the quasi-definite KKT matrix
// must have n positive pivots, which holds iff P + sigma I + A' diag(rho) A is positive
// definite -- the reduced matrix the solve kernels factor): one factor-only launch of the
// solve kernel per shard, which stops after the first factorisation and marks an instance
// whose factorisation fails as non-convex.  The first such instance is reported.
// The setup's invalid-data flags (check_err_flags) and osqp_setup's convexity test
// (check_convex) behind the setup kernel with one synchronisation: the factor-only launch is
// enqueued right after it, and both the flags and the statuses come back through the shard's
// pinned staging (update()'s, allocated here) in stream order.  Invalid data is reported
// first, as the two checks in turn would.
int check_setup(mpcqp_handle* h) {
    const long n = h->n, m = h->m;
    std::vector<int*> got(h->shards.size(), nullptr);
    std::vector<std::vector<int>> host(h->shards.size());
    std::vector<long> stoff(h->shards.size(), 0);  // status's offset from err in got[]
    for (size_t si = 0; si < h->shards.size(); ++si) {
        Shard& s = h->shards[si];
        HIPCHK(hipSetDevice(s.dev));
        if (int e = stream_enter(s, s.stream)) return e;
        HIPCHK(launch_solve(s.kp, s.B, s.out_x, s.out_y, 1, s.stream));
        // err and status in one copy: the workspace carves err right before status
        const size_t span = (size_t)((const char*)(s.kp.status + s.B) - (const char*)s.kp.err);
        const size_t ib = std::max(span, sizeof(double) * (size_t)s.B * (n + 2 * m) + sizeof(int) * (size_t)s.B);
        if (ib <= kStageMax) {
            if (!s.hin) {
                HIPCHK(pool_malloc(s.dev, ib, (void**)&s.hin, true));
                s.hin_bytes = ib;
            }
            got[si] = (int*)s.hin;  // err (B), then status (B) at stoff[si]
            HIPCHK(hipMemcpyAsync(got[si], s.kp.err, span, hipMemcpyDeviceToHost, s.stream));
            stoff[si] = s.kp.status - s.kp.err;
        }
        if (int e = stream_leave(s, s.stream)) return e;
    }
    if (int e = sync_all(h)) return e;
    for (size_t si = 0; si < h->shards.size(); ++si) {
        Shard& s = h->shards[si];
        if (!got[si]) {
            host[si].resize(2 * s.B);
            HIPCHK(hipSetDevice(s.dev));
            HIPCHK(hipMemcpy(host[si].data(), s.kp.err, sizeof(int) * s.B, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(host[si].data() + s.B, s.kp.status, sizeof(int) * s.B, hipMemcpyDeviceToHost));
            got[si] = host[si].data();
            stoff[si] = s.B;
        }
    }
    for (size_t si = 0; si < h->shards.size(); ++si)
        for (long i = 0; i < h->shards[si].B; ++i)
            if (got[si][i])
                return fail(MPCQP_EINVAL, "instance %ld: invalid data (l > u or NaN bounds)", h->shards[si].b0 + i);
    for (size_t si = 0; si < h->shards.size(); ++si)
        for (long i = 0; i < h->shards[si].B; ++i)
            if (got[si][stoff[si] + i] == MPCQP_NON_CVX_)
                return fail(MPCQP_ENONCVX, "instance %ld: P is not convex (the KKT matrix is not quasi-definite)",
                            h->shards[si].b0 + i);
    return 0;
}

int check_convex(mpcqp_handle* h) {
    for (auto& s : h->shards) {
        HIPCHK(hipSetDevice(s.dev));
        if (int e = stream_enter(s, s.stream)) return e;
        HIPCHK(launch_solve(s.kp, s.B, s.out_x, s.out_y, 1, s.stream));
        if (int e = stream_leave(s, s.stream)) return e;
    }
    if (int e = sync_all(h)) return e;
    for (auto& s : h->shards) {
        std::vector<int> st(s.B);
        HIPCHK(hipSetDevice(s.dev));
        HIPCHK(hipMemcpy(st.data(), s.kp.status, sizeof(int) * s.B, hipMemcpyDeviceToHost));
        for (long i = 0; i < s.B; ++i)
            if (st[i] == MPCQP_NON_CVX_)
                return fail(MPCQP_ENONCVX, "instance %ld: P is not convex (the KKT matrix is not quasi-definite)",
                            s.b0 + i);
    }
    return 0;
}

void free_shard(Shard& s) {
    (void)hipSetDevice(s.dev);
    if (s.stream) (void)hipStreamSynchronize(s.stream);
    if (s.last_st && s.last_st != s.stream && s.last_ev)
        (void)hipEventSynchronize(s.last_ev);  // a caller stream's last call
    pool_free(s.dev, s.dws_bytes, s.dws, false);
    pool_free(s.dev, s.dplan_bytes, s.dplan, false, s.dplan_tag);
    pool_free(s.dev, s.hstage_bytes, s.hstage, true);
    pool_free(s.dev, s.dstage_bytes, s.dstage, false);
    pool_free(s.dev, s.hin_bytes, s.hin, true);
    pool_stream_release(s);
    s = Shard{};
}

// Move a handle whose plan eliminated variables (choose_plan: the slack layouts) onto the
// plain plan, keeping its state, so that polish -- whose factorisation covers all of K
// (factorize<POL>) -- can run (osqp-python's update_settings(polish=True) at any time).
// Everything a solve carries from call to call moves over unchanged: the scaled data and
// the scaling, the iterates x, z, y, each instance's rho and row classes, its last status,
// info and certificates, the setup inputs; the per-column arrays (q, D, x: padded order)
// are permuted from the old padded index to the new one, and the scaled A values from the
// old plan's padded-CSC order to the new one's.  The factor is formed at the start
// of every solve, so nothing of it is kept.  The dispatch order restarts in identity order.
int replan_plain(mpcqp_handle* h) {
    if (int e = sync_all(h)) return e;
    mpcqp_settings st = h->set;
    st.polish = 1;
    auto npl = std::make_shared<Plan>();
    std::string err = choose_plan(h->n, h->m, h->Pp.data(), h->Pi.data(), h->Ap.data(), h->Ai.data(), st, *npl);
    if (!err.empty()) return fail(MPCQP_EUNSUPPORTED, "re-plan for polish: %s", err.c_str());
    std::shared_ptr<const Plan> oldp = h->plan;
    const Plan& old = *oldp;
    h->plan = npl;
    const long n = h->n, m = h->m, npo = old.npad, npn = h->plan->npad;
    std::vector<Shard> fresh;
    int rc = 0;
    for (auto& os : h->shards) {
        Shard s;
        s.dev = os.dev; s.b0 = os.b0; s.B = os.B;
        fresh.push_back(s);
        if ((rc = alloc_shard(h, fresh.back(), os.in_Px != nullptr))) break;
        Shard& ns = fresh.back();
        KParams &a = os.kp, &b = ns.kp;
        b.mat_shared = a.mat_shared;
        b.polish = a.polish; b.refine_iter = a.refine_iter; b.delta = a.delta;
        b.alpha = a.alpha; b.eps_abs = a.eps_abs; b.eps_rel = a.eps_rel; b.eps_pinf = a.eps_pinf;
        b.eps_dinf = a.eps_dinf; b.rho0 = a.rho0; b.max_iter = a.max_iter; b.check_term = a.check_term;
        b.warm_start = a.warm_start; b.scaled_term = a.scaled_term;
        const long B = s.B;
        auto cp = [&](void* d, const void* src, size_t bytes) -> int {
            if (bytes) HIPCHK(hipMemcpy(d, src, bytes, hipMemcpyDeviceToDevice));
            return 0;
        };
        const size_t D8 = sizeof(double), I4 = sizeof(int);
        if ((rc = cp(b.Px, a.Px, D8 * B * old.nnzP)) ||
            (rc = cp(b.l, a.l, D8 * B * m)) || (rc = cp(b.u, a.u, D8 * B * m)) || (rc = cp(b.E, a.E, D8 * B * m)) ||
            (rc = cp(b.z, a.z, D8 * B * m)) || (rc = cp(b.y, a.y, D8 * B * m)) || (rc = cp(b.scal, a.scal, D8 * B * 4)) ||
            (rc = cp(b.dyc, a.dyc, D8 * B * m)) || (rc = cp(b.dxc, a.dxc, D8 * B * n)) ||
            (rc = cp(b.obj, a.obj, D8 * B)) || (rc = cp(b.pri, a.pri, D8 * B)) || (rc = cp(b.dua, a.dua, D8 * B)) ||
            (rc = cp(b.rho_est, a.rho_est, D8 * B)) || (rc = cp(b.ct, a.ct, (size_t)B * m)) ||
            (rc = cp(b.status, a.status, I4 * B)) || (rc = cp(b.iter, a.iter, I4 * B)) ||
            (rc = cp(b.rho_upd, a.rho_upd, I4 * B)) || (rc = cp(b.pstat, a.pstat, I4 * B)) ||
            (rc = cp(b.err, a.err, I4 * B)))
            break;
        if (os.in_Px &&
            ((rc = cp(ns.in_Px, os.in_Px, D8 * B * old.nnzP)) || (rc = cp(ns.in_Ax, os.in_Ax, D8 * B * old.nnzA)) ||
             (rc = cp(ns.in_q, os.in_q, D8 * B * n)) || (rc = cp(ns.in_l, os.in_l, D8 * B * m)) ||
             (rc = cp(ns.in_u, os.in_u, D8 * B * m)) || (rc = cp(ns.out_x, os.out_x, D8 * B * n)) ||
             (rc = cp(ns.out_y, os.out_y, D8 * B * m))))
            break;
        // q, D, x: padded order -> the new padded order (padding: q = 0, D = 1, x = 0, as setup leaves it)
        double* cols_old[3] = {a.q, a.D, a.x};
        double* cols_new[3] = {b.q, b.D, b.x};
        std::vector<double> ho((size_t)B * npo), hn((size_t)B * npn);
        for (int t = 0; t < 3 && !rc; ++t) {
            if (hipMemcpy(ho.data(), cols_old[t], D8 * B * npo, hipMemcpyDeviceToHost) != hipSuccess) {
                rc = fail(MPCQP_EDEVICE, "re-plan: copy-out failed");
                break;
            }
            std::fill(hn.begin(), hn.end(), t == 1 ? 1.0 : 0.0);
            for (long i = 0; i < B; ++i)
                for (long j = 0; j < n; ++j) hn[i * npn + h->plan->var_pad[j]] = ho[i * npo + old.var_pad[j]];
            if (hipMemcpy(cols_new[t], hn.data(), D8 * B * npn, hipMemcpyHostToDevice) != hipSuccess)
                rc = fail(MPCQP_EDEVICE, "re-plan: copy-in failed");
        }
        // the scaled A values: the padded-CSC order of each plan (k.Ax[e] = Ax[acsc_v[e]],
        // kernels.hip::k_setup), user value v at csc_pos[v]
        if (!rc && old.nnzA > 0) {
            const long nz = old.nnzA;
            std::vector<double> ao((size_t)B * nz), an((size_t)B * nz);
            if (hipMemcpy(ao.data(), a.Ax, D8 * B * nz, hipMemcpyDeviceToHost) != hipSuccess) {
                rc = fail(MPCQP_EDEVICE, "re-plan: copy-out failed");
            } else {
                for (long i = 0; i < B; ++i)
                    for (long v = 0; v < nz; ++v) an[i * nz + h->plan->csc_pos[v]] = ao[i * nz + old.csc_pos[v]];
                if (hipMemcpy(b.Ax, an.data(), D8 * B * nz, hipMemcpyHostToDevice) != hipSuccess)
                    rc = fail(MPCQP_EDEVICE, "re-plan: copy-in failed");
            }
        }
        if (rc) break;
        (void)hipSetDevice(ns.dev);
        if (hipMemcpy((void*)b.self, &b, sizeof(KParams), hipMemcpyHostToDevice) != hipSuccess) {
            rc = fail(MPCQP_EDEVICE, "re-plan: parameter copy failed");
            break;
        }
    }
    if (rc) {  // the handle keeps its old plan and workspace
        for (auto& s : fresh) free_shard(s);
        h->plan = oldp;
        return rc;
    }
    for (auto& s : h->shards) free_shard(s);
    h->shards.swap(fresh);
    h->staged = false;
    return 0;
}

}  // namespace

extern "C" {

void mpcqp_default_settings(mpcqp_settings* s) {
    s->rho = 0.1; s->sigma = 1e-6; s->alpha = 1.6;
    s->eps_abs = 1e-3; s->eps_rel = 1e-3; s->eps_prim_inf = 1e-4; s->eps_dual_inf = 1e-4;
    s->adaptive_rho_tolerance = 5.0;
    s->max_iter = 4000; s->scaling = 10; s->check_termination = 25; s->warm_start = 1;
    s->adaptive_rho = 1; s->adaptive_rho_interval = 0; s->scaled_termination = 0; s->polish = 0;
    s->verbose = 0; s->delta = 1e-6; s->polish_refine_iter = 3;
}

const char* mpcqp_last_error(void) { return g_err.c_str(); }

int mpcqp_analyze(int32_t n, int32_t m, const int32_t* Pp, const int32_t* Pi, const int32_t* Ap,
                  const int32_t* Ai, int32_t* nb, int32_t* block, int32_t* var_pad, int32_t* bsize) {
    return mpcqp_analyze_ex(n, m, Pp, Pi, Ap, Ai, 0, nb, block, var_pad, bsize, nullptr);
}

int mpcqp_analyze_ex(int32_t n, int32_t m, const int32_t* Pp, const int32_t* Pi, const int32_t* Ap,
                     const int32_t* Ai, int32_t eliminate, int32_t* nb, int32_t* block, int32_t* var_pad,
                     int32_t* bsize, int32_t* n_eliminated) {
    Plan pl;
    std::string err = build_plan(n, m, Pp, Pi, Ap, Ai, pl, eliminate != 0, !eliminate);
    if (n_eliminated) *n_eliminated = pl.ne;
    if (!err.empty()) return fail(err.rfind("unsupported", 0) == 0 ? MPCQP_EUNSUPPORTED : MPCQP_EINVAL, "%s", err.c_str());
    if (nb) *nb = pl.nb;
    if (block) *block = kS;
    if (var_pad) std::copy(pl.var_pad.begin(), pl.var_pad.end(), var_pad);
    if (bsize) std::copy(pl.bsize.begin(), pl.bsize.end(), bsize);
    return 0;
}

int mpcqp_setup_batch(int32_t n, int32_t m, const int32_t* Pp, const int32_t* Pi, const int32_t* Ap,
                      const int32_t* Ai, int64_t B, const double* Px, const double* Ax, const double* q,
                      const double* l, const double* u, const mpcqp_settings* settings,
                      uint32_t device_mask, mpcqp_handle** out) {
    if (!Px || !Ax || !q || !l || !u) return fail(MPCQP_EINVAL, "NULL data array");
    std::vector<int> devs;
    for (int d = 0; d < 32; ++d)
        if (device_mask & (1u << d)) devs.push_back(d);
    if (devs.empty()) devs.push_back(0);
    // MPCQP_SPLIT=k (diagnostic): k contiguous shards per selected device, each with its own
    // stream, workspace and dispatch order -- the multi-device shard / gather code (b0
    // offsets, launch-all-then-gather) exercised on a one-GPU box
    if (const char* ev = getenv("MPCQP_SPLIT"); ev && atoi(ev) > 1) {
        const int k = std::min(atoi(ev), 64);
        std::vector<int> rep;
        for (int d : devs)
            for (int i = 0; i < k; ++i) rep.push_back(d);
        devs.swap(rep);
    }
    mpcqp_handle* h = nullptr;
    if (int e = make_handle(n, m, Pp, Pi, Ap, Ai, B, settings, devs, true, &h)) return e;
    if (int e = check_bounds_host(h, l, u, B)) { mpcqp_free(h); return e; }
    const Plan& pl = *h->plan;
    auto upload = [&](Shard& s) -> int {
        const long b0 = s.b0, Bs = s.B;
        HIPCHK(hipSetDevice(s.dev));
        // the five inputs lie one after another in the workspace (alloc_shard's carve): a small
        // shard stages them in pinned memory with the same layout and goes up in one copy (five
        // pageable copies cost ~4 us each on a one-QP setup)
        const size_t span = (size_t)((const char*)(s.in_u + Bs * m) - (const char*)s.in_Px);
        const size_t upd = sizeof(double) * (size_t)Bs * (n + 2 * m) + sizeof(int) * (size_t)Bs;  // (update's use)
        if (span <= kStageMax) {
            if (!s.hin) {
                HIPCHK(pool_malloc(s.dev, std::max(span, upd), (void**)&s.hin, true));
                s.hin_bytes = std::max(span, upd);
            }
            char* const hb = (char*)s.hin;
            auto put = [&](const double* dst, const double* src, size_t cnt) {
                memcpy(hb + ((const char*)dst - (const char*)s.in_Px), src, sizeof(double) * cnt);
            };
            put(s.in_Px, Px + b0 * pl.nnzP, (size_t)Bs * pl.nnzP);
            put(s.in_Ax, Ax + b0 * pl.nnzA, (size_t)Bs * pl.nnzA);
            put(s.in_q, q + b0 * n, (size_t)Bs * n);
            put(s.in_l, l + b0 * m, (size_t)Bs * m);
            put(s.in_u, u + b0 * m, (size_t)Bs * m);
            HIPCHK(hipMemcpyAsync(s.in_Px, hb, span, hipMemcpyHostToDevice, s.stream));
        } else {
            HIPCHK(hipMemcpyAsync(s.in_Px, Px + b0 * pl.nnzP, sizeof(double) * Bs * pl.nnzP, hipMemcpyHostToDevice, s.stream));
            HIPCHK(hipMemcpyAsync(s.in_Ax, Ax + b0 * pl.nnzA, sizeof(double) * Bs * pl.nnzA, hipMemcpyHostToDevice, s.stream));
            HIPCHK(hipMemcpyAsync(s.in_q, q + b0 * n, sizeof(double) * Bs * n, hipMemcpyHostToDevice, s.stream));
            HIPCHK(hipMemcpyAsync(s.in_l, l + b0 * m, sizeof(double) * Bs * m, hipMemcpyHostToDevice, s.stream));
            HIPCHK(hipMemcpyAsync(s.in_u, u + b0 * m, sizeof(double) * Bs * m, hipMemcpyHostToDevice, s.stream));
        }
        HIPCHK(launch_setup(s.kp, Bs, s.in_Px, s.in_Ax, s.in_q, s.in_l, s.in_u, s.stream));
        return stream_leave(s, s.stream);
    };
    strace().mark("handle");
    for (auto& s : h->shards)
        if (int e = upload(s)) { mpcqp_free(h); return e; }
    strace().mark("inputs + setup launch");
    if (int e = check_setup(h)) { mpcqp_free(h); return e; }
    strace().mark("setup + convexity wait");
    *out = h;
    return 0;
}

int mpcqp_update_batch(mpcqp_handle* h, const double* q, const double* l, const double* u) {
    if (int e = need_state(h, "mpcqp_update_batch")) return e;
    if (!h) return fail(MPCQP_EINVAL, "NULL handle");
    h->staged = false;  // (device work: the staged results of the last solve are stale)
    if (l && u)
        if (int e = check_bounds_host(h, l, u, h->B)) return e;
    const long n = h->n, m = h->m;
    // small shards go through pinned staging: the copies and the error flags' read-back are
    // asynchronous and the call synchronises once (osqp's per-step update of one problem)
    auto in_bytes = [&](long Bs) { return sizeof(double) * (size_t)Bs * (n + 2 * m) + sizeof(int) * (size_t)Bs; };
    for (auto& s : h->shards) {
        HIPCHK(hipSetDevice(s.dev));
        if (int e = stream_enter(s, s.stream)) return e;
        const long Bs = s.B;
        if (in_bytes(Bs) <= kStageMax) {
            if (!s.hin) {
                HIPCHK(pool_malloc(s.dev, in_bytes(Bs), (void**)&s.hin, true));
                s.hin_bytes = in_bytes(Bs);
            }
            double *hq = (double*)s.hin, *hl = hq + Bs * n, *hu = hl + Bs * m;
            int* herr = (int*)(hu + Bs * m);
            if (q) {
                std::copy(q + s.b0 * n, q + (s.b0 + Bs) * n, hq);
                HIPCHK(hipMemcpyAsync(s.in_q, hq, sizeof(double) * Bs * n, hipMemcpyHostToDevice, s.stream));
            }
            if (l) {
                std::copy(l + s.b0 * m, l + (s.b0 + Bs) * m, hl);
                HIPCHK(hipMemcpyAsync(s.in_l, hl, sizeof(double) * Bs * m, hipMemcpyHostToDevice, s.stream));
            }
            if (u) {
                std::copy(u + s.b0 * m, u + (s.b0 + Bs) * m, hu);
                HIPCHK(hipMemcpyAsync(s.in_u, hu, sizeof(double) * Bs * m, hipMemcpyHostToDevice, s.stream));
            }
            HIPCHK(launch_update(s.kp, Bs, q ? s.in_q : nullptr, l ? s.in_l : nullptr, u ? s.in_u : nullptr, s.stream));
            if (l || u) HIPCHK(hipMemcpyAsync(herr, s.kp.err, sizeof(int) * Bs, hipMemcpyDeviceToHost, s.stream));
        } else {
            if (q) HIPCHK(hipMemcpyAsync(s.in_q, q + s.b0 * n, sizeof(double) * Bs * n, hipMemcpyHostToDevice, s.stream));
            if (l) HIPCHK(hipMemcpyAsync(s.in_l, l + s.b0 * m, sizeof(double) * Bs * m, hipMemcpyHostToDevice, s.stream));
            if (u) HIPCHK(hipMemcpyAsync(s.in_u, u + s.b0 * m, sizeof(double) * Bs * m, hipMemcpyHostToDevice, s.stream));
            HIPCHK(launch_update(s.kp, Bs, q ? s.in_q : nullptr, l ? s.in_l : nullptr, u ? s.in_u : nullptr, s.stream));
        }
        if (int e = stream_leave(s, s.stream)) return e;
    }
    if (int e = sync_all(h)) return e;
    if (!(l || u)) return 0;
    for (auto& s : h->shards) {
        if (in_bytes(s.B) > kStageMax) {
            std::vector<int> err(s.B);
            HIPCHK(hipSetDevice(s.dev));
            HIPCHK(hipMemcpy(err.data(), s.kp.err, sizeof(int) * s.B, hipMemcpyDeviceToHost));
            for (long i = 0; i < s.B; ++i)
                if (err[i]) return fail(MPCQP_EINVAL, "instance %ld: invalid data (l > u or NaN bounds)", s.b0 + i);
        } else {
            const int* herr = (const int*)((const double*)s.hin + s.B * (n + 2 * m));
            for (long i = 0; i < s.B; ++i)
                if (herr[i]) return fail(MPCQP_EINVAL, "instance %ld: invalid data (l > u or NaN bounds)", s.b0 + i);
        }
    }
    return 0;
}

int mpcqp_update_matrices_batch(mpcqp_handle* h, const double* Px, const int32_t* Px_idx, int32_t nPx,
                                const double* Ax, const int32_t* Ax_idx, int32_t nAx) {
    if (int e = need_state(h, "mpcqp_update_matrices_batch")) return e;
    if (!h) return fail(MPCQP_EINVAL, "NULL handle");
    h->staged = false;  // (device work: the staged results of the last solve are stale)
    if (!Px && !Ax) return fail(MPCQP_EINVAL, "no matrix values given");
    const Plan& pl = *h->plan;
    // the columns of the value arrays that are written: all, or per index its last
    // occurrence (OSQP's sequential loop: a repeated index takes the last value)
    auto pick_cols = [&](const int32_t* idx, int32_t k, int nnz, const char* name, std::vector<int>& col,
                         std::vector<int>& dst) -> int {
        if (!idx) {
            col.resize(nnz);
            for (int i = 0; i < nnz; ++i) col[i] = i;
            dst = col;
            return 0;
        }
        if (k < 0 || k > nnz)
            return fail(MPCQP_EINVAL, "new number of elements (%d) greater than elements in %s (%d)", k, name, nnz);
        std::vector<int> last(nnz, -1);
        for (int i = 0; i < k; ++i) {
            if (idx[i] < 0 || idx[i] >= nnz) return fail(MPCQP_EINVAL, "%s index %d out of range", name, idx[i]);
            last[idx[i]] = i;
        }
        for (int v = 0; v < nnz; ++v)
            if (last[v] >= 0) { col.push_back(last[v]); dst.push_back(v); }
        return 0;
    };
    std::vector<int> pcol, pdst, acol, adst;
    if (Px)
        if (int e = pick_cols(Px_idx, nPx, pl.nnzP, "P", pcol, pdst)) return e;
    if (Ax)
        if (int e = pick_cols(Ax_idx, nAx, pl.nnzA, "A", acol, adst)) return e;
    const int kP = Px ? (Px_idx ? nPx : pl.nnzP) : 0, kA = Ax ? (Ax_idx ? nAx : pl.nnzA) : 0;
    const int nP = (int)pdst.size(), nA = (int)adst.size();
    for (auto& s : h->shards) {
        if (!s.in_Px) return fail(MPCQP_EINVAL, "matrix updates need a handle made by mpcqp_setup_batch");
        if (s.kp.mat_shared) return fail(MPCQP_EINVAL, "matrix updates need per-instance matrices (shared mode is on)");
    }
    // per shard: the selected values (Bs x nP, Bs x nA) and their indices, in one staging
    // allocation freed after the call
    std::vector<void*> tmp(h->shards.size(), nullptr);
    auto release = [&]() {
        for (size_t i = 0; i < tmp.size(); ++i)
            if (tmp[i]) { (void)hipSetDevice(h->shards[i].dev); (void)hipFree(tmp[i]); }
    };
    int err = 0;
    std::vector<std::vector<double>> host(h->shards.size());
    for (size_t si = 0; si < h->shards.size() && !err; ++si) {
        Shard& s = h->shards[si];
        const long Bs = s.B;
        std::vector<double>& hv = host[si];
        hv.resize((size_t)Bs * (nP + nA));
        for (long b = 0; b < Bs; ++b) {
            for (int k = 0; k < nP; ++k) hv[b * nP + k] = Px[(s.b0 + b) * kP + pcol[k]];
            for (int k = 0; k < nA; ++k) hv[Bs * nP + b * nA + k] = Ax[(s.b0 + b) * kA + acol[k]];
        }
        const size_t vbytes = sizeof(double) * hv.size(), ibytes = sizeof(int) * (size_t)(nP + nA);
        auto step = [&]() -> int {
            HIPCHK(hipSetDevice(s.dev));
            HIPCHK(hipMalloc(&tmp[si], vbytes + ibytes + 16));
            double* dv = (double*)tmp[si];
            int* di = (int*)((char*)tmp[si] + vbytes);
            if (int e = stream_enter(s, s.stream)) return e;
            if (vbytes) HIPCHK(hipMemcpyAsync(dv, hv.data(), vbytes, hipMemcpyHostToDevice, s.stream));
            if (nP) HIPCHK(hipMemcpyAsync(di, pdst.data(), sizeof(int) * nP, hipMemcpyHostToDevice, s.stream));
            if (nA) HIPCHK(hipMemcpyAsync(di + nP, adst.data(), sizeof(int) * nA, hipMemcpyHostToDevice, s.stream));
            HIPCHK(launch_update_mat(s.kp, Bs, s.in_Px, s.in_Ax, s.in_q, s.in_l, s.in_u, Px ? dv : nullptr, di, nP,
                                     Ax ? dv + Bs * nP : nullptr, di + nP, nA, s.stream));
            return stream_leave(s, s.stream);
        };
        err = step();
    }
    if (!err) err = sync_all(h);
    release();
    if (err) return err;
    if (int e = check_err_flags(h)) return e;
    return check_convex(h);  // osqp_update_P_A refactors at once and reports a failed factorisation
}

int mpcqp_update_settings(mpcqp_handle* h, const mpcqp_settings* s, int32_t set_rho) {
    if (!h || !s) return fail(MPCQP_EINVAL, "NULL argument");
    h->staged = false;  // (device work: the staged results of the last solve are stale)
    const mpcqp_settings& o = h->set;
    if (s->sigma != o.sigma || s->scaling != o.scaling || s->adaptive_rho != o.adaptive_rho ||
        s->adaptive_rho_tolerance != o.adaptive_rho_tolerance || s->adaptive_rho_interval != o.adaptive_rho_interval)
        return fail(MPCQP_EINVAL, "sigma, scaling and the adaptive-rho settings cannot be changed after setup");
    if (int e = validate_settings(*s)) return e;  // (polish's delta / refinement steps included)
    if (s->polish && h->plan->ne > 0)  // polish factors all of K: the plain plan, state kept
        if (int e = replan_plain(h)) return e;
    const bool rho_changed = set_rho != 0;
    const double rho = std::min(std::max(s->rho, 1e-6), 1e6);  // osqp_update_rho: RHO_MIN / RHO_MAX
    for (auto& sh : h->shards) {
        KParams& k = sh.kp;
        k.alpha = s->alpha; k.eps_abs = s->eps_abs; k.eps_rel = s->eps_rel;
        k.eps_pinf = s->eps_prim_inf; k.eps_dinf = s->eps_dual_inf; k.rho0 = s->rho;
        k.max_iter = s->max_iter; k.check_term = s->check_termination; k.warm_start = s->warm_start;
        k.scaled_term = s->scaled_termination; k.polish = s->polish; k.refine_iter = s->polish_refine_iter;
        k.delta = s->delta;
        // (rho_interval keeps the value setup resolved: OSQP resolves the automatic interval
        // in osqp_setup, so check_termination set later does not move it)
        HIPCHK(hipSetDevice(sh.dev));
        if (int e = stream_enter(sh, sh.stream)) return e;
        HIPCHK(hipMemcpyAsync((void*)k.self, &k, sizeof(KParams), hipMemcpyHostToDevice, sh.stream));
        if (rho_changed) {  // every instance's current rho (scal[2]); the solve refactors with it
            HIPCHK(hipMemsetAsync(k.ffresh, 0, sizeof(int) * sh.B, sh.stream));
            std::vector<double> r(sh.B, rho);
            HIPCHK(hipMemcpy2DAsync(k.scal + 2, 4 * sizeof(double), r.data(), sizeof(double), sizeof(double), sh.B,
                                    hipMemcpyHostToDevice, sh.stream));
            HIPCHK(hipStreamSynchronize(sh.stream));  // r is a host temporary
        }
        if (int e = stream_leave(sh, sh.stream)) return e;
    }
    const int interval = h->set.adaptive_rho_interval;
    h->set = *s;
    h->set.adaptive_rho_interval = interval;
    return sync_all(h);
}

int mpcqp_warm_start_batch(mpcqp_handle* h, const double* x, const double* y) {
    if (int e = need_state(h, "mpcqp_warm_start_batch")) return e;
    if (!h) return fail(MPCQP_EINVAL, "NULL handle");
    h->staged = false;  // (device work: the staged results of the last solve are stale)
    const long n = h->n, m = h->m;
    for (auto& s : h->shards) {
        HIPCHK(hipSetDevice(s.dev));
        if (int e = stream_enter(s, s.stream)) return e;
        if (x) HIPCHK(hipMemcpyAsync(s.out_x, x + s.b0 * n, sizeof(double) * s.B * n, hipMemcpyHostToDevice, s.stream));
        if (y) HIPCHK(hipMemcpyAsync(s.out_y, y + s.b0 * m, sizeof(double) * s.B * m, hipMemcpyHostToDevice, s.stream));
        HIPCHK(launch_warm(s.kp, s.B, x ? s.out_x : nullptr, y ? s.out_y : nullptr, s.stream));
        if (int e = stream_leave(s, s.stream)) return e;
        s.kp.warm_start = 1;
    }
    h->set.warm_start = 1;
    return sync_all(h);
}

int mpcqp_solve_batch(mpcqp_handle* h, double* x, double* y, int32_t* status, int32_t* iters) {
    if (int e = need_state(h, "mpcqp_solve_batch")) return e;
    if (!h) return fail(MPCQP_EINVAL, "NULL handle");
    const long n = h->n, m = h->m;
    // every shard's kernels are enqueued before any result is copied back: a copy into the
    // caller's (pageable) memory blocks the host until its shard is done, so copying inside
    // the launch loop would start shard d+1 only after shard d had finished
    // an event pair around the solve launch only while timing is on (mpcqp_timing): two event
    // packets cost a one-QP solve() ~5.5 us of its ~150 (cfg 2, same-box A/B, profiles/r6/lat_events_ab.txt)
    const bool evs = h->collect;
    for (auto& s : h->shards) {
        HIPCHK(hipSetDevice(s.dev));
        if (int e = stream_enter(s, s.stream)) return e;
        if (evs) HIPCHK(hipEventRecord(s.ev0, s.stream));
        HIPCHK(launch_solve(s.kp, s.B, s.out_x, s.out_y, 0, s.stream));
        if (evs) HIPCHK(hipEventRecord(s.ev1, s.stream));
        HIPCHK(launch_order(s.kp, s.B, s.stream));
        if (int e = stream_leave(s, s.stream)) return e;
    }
    // the host-side gather: each shard's slice of the caller's buffers, in shard order; a
    // small shard stages everything its solve returns in pinned memory (one synchronisation
    // for the solve and the getters that follow it, instead of one per array)
    bool all_staged = true;
    for (auto& s : h->shards) {
        HIPCHK(hipSetDevice(s.dev));
        const size_t sb = stage_bytes(h, s.B);
        if (sb <= kStageMax) {
            if (!s.hstage) {
                HIPCHK(pool_malloc(s.dev, sb, (void**)&s.hstage, true));
                s.hstage_bytes = sb;
            }
            if (!s.dstage) {
                HIPCHK(pool_malloc(s.dev, sb, (void**)&s.dstage, false));
                s.dstage_bytes = sb;
            }
            const Stage g = stage_of(h, s);
            const long Bs = s.B;
            // one gather kernel into the device twin of the staging layout, one copy down
            GatherList gl{};
            auto add = [&](const void* hdst, const void* src, long cnt, int sz) {
                GatherSeg& e = gl.seg[gl.nseg++];
                e.src = src;
                e.off = (long)((const char*)hdst - s.hstage);
                e.cnt = cnt;
                e.sz = sz;
                gl.most = std::max(gl.most, cnt);
            };
            add(g.x, s.out_x, Bs * n, 8);
            add(g.y, s.out_y, Bs * m, 8);
            add(g.obj, s.kp.obj, Bs, 8);
            add(g.pri, s.kp.pri, Bs, 8);
            add(g.dua, s.kp.dua, Bs, 8);
            add(g.rho_est, s.kp.rho_est, Bs, 8);
            add(g.dxc, s.kp.dxc, Bs * n, 8);
            add(g.dyc, s.kp.dyc, Bs * m, 8);
            add(g.status, s.kp.status, Bs, 4);
            add(g.iter, s.kp.iter, Bs, 4);
            add(g.rho_upd, s.kp.rho_upd, Bs, 4);
            add(g.pstat, h->set.polish ? (const void*)s.kp.pstat : nullptr, Bs, 4);  // (no polish: zeros)
            HIPCHK(launch_gather(gl, s.dstage, s.stream));
            HIPCHK(hipMemcpyAsync(s.hstage, s.dstage, sb, hipMemcpyDeviceToHost, s.stream));
        } else {
            all_staged = false;
            if (x) HIPCHK(hipMemcpyAsync(x + s.b0 * n, s.out_x, sizeof(double) * s.B * n, hipMemcpyDeviceToHost, s.stream));
            if (y) HIPCHK(hipMemcpyAsync(y + s.b0 * m, s.out_y, sizeof(double) * s.B * m, hipMemcpyDeviceToHost, s.stream));
            if (status) HIPCHK(hipMemcpyAsync(status + s.b0, s.kp.status, sizeof(int) * s.B, hipMemcpyDeviceToHost, s.stream));
            if (iters) HIPCHK(hipMemcpyAsync(iters + s.b0, s.kp.iter, sizeof(int) * s.B, hipMemcpyDeviceToHost, s.stream));
        }
    }
    if (int e = sync_all(h)) return e;
    for (auto& s : h->shards) {
        if (stage_bytes(h, s.B) > kStageMax) continue;
        const Stage g = stage_of(h, s);
        if (x) std::copy(g.x, g.x + s.B * n, x + s.b0 * n);
        if (y) std::copy(g.y, g.y + s.B * m, y + s.b0 * m);
        if (status) std::copy(g.status, g.status + s.B, status + s.b0);
        if (iters) std::copy(g.iter, g.iter + s.B, iters + s.b0);
    }
    h->staged = all_staged;
    float ms = 0.f;
    h->last_ms = -1.0;
    if (evs && h->shards.size() == 1 && hipEventElapsedTime(&ms, h->shards[0].ev0, h->shards[0].ev1) == hipSuccess) {
        h->last_ms = ms;
        h->last_pair = {h->shards[0].ev0, h->shards[0].ev1};
    }
    return 0;
}

int mpcqp_get_info_batch(mpcqp_handle* h, double* obj_val, double* pri_res, double* dua_res,
                         double* rho_estimate, int32_t* rho_updates) {
    if (!h) return fail(MPCQP_EINVAL, "NULL handle");
    if (h->staged) {
        for (auto& s : h->shards) {
            const Stage g = stage_of(h, s);
            if (obj_val) std::copy(g.obj, g.obj + s.B, obj_val + s.b0);
            if (pri_res) std::copy(g.pri, g.pri + s.B, pri_res + s.b0);
            if (dua_res) std::copy(g.dua, g.dua + s.B, dua_res + s.b0);
            if (rho_estimate) std::copy(g.rho_est, g.rho_est + s.B, rho_estimate + s.b0);
            if (rho_updates) std::copy(g.rho_upd, g.rho_upd + s.B, rho_updates + s.b0);
        }
        return 0;
    }
    for (auto& s : h->shards) {
        HIPCHK(hipSetDevice(s.dev));
        if (obj_val) HIPCHK(hipMemcpy(obj_val + s.b0, s.kp.obj, sizeof(double) * s.B, hipMemcpyDeviceToHost));
        if (pri_res) HIPCHK(hipMemcpy(pri_res + s.b0, s.kp.pri, sizeof(double) * s.B, hipMemcpyDeviceToHost));
        if (dua_res) HIPCHK(hipMemcpy(dua_res + s.b0, s.kp.dua, sizeof(double) * s.B, hipMemcpyDeviceToHost));
        if (rho_estimate) HIPCHK(hipMemcpy(rho_estimate + s.b0, s.kp.rho_est, sizeof(double) * s.B, hipMemcpyDeviceToHost));
        if (rho_updates) HIPCHK(hipMemcpy(rho_updates + s.b0, s.kp.rho_upd, sizeof(int) * s.B, hipMemcpyDeviceToHost));
    }
    return 0;
}

int mpcqp_get_polish_status(mpcqp_handle* h, int32_t* status_polish) {
    if (!h || !status_polish) return fail(MPCQP_EINVAL, "NULL argument");
    if (h->staged) {
        for (auto& s : h->shards) {
            const Stage g = stage_of(h, s);
            std::copy(g.pstat, g.pstat + s.B, status_polish + s.b0);
        }
        return 0;
    }
    for (auto& s : h->shards) {
        HIPCHK(hipSetDevice(s.dev));
        if (h->set.polish)
            HIPCHK(hipMemcpy(status_polish + s.b0, s.kp.pstat, sizeof(int) * s.B, hipMemcpyDeviceToHost));
        else
            std::fill(status_polish + s.b0, status_polish + s.b0 + s.B, 0);
    }
    return 0;
}

int mpcqp_get_certificates(mpcqp_handle* h, double* prim_inf_cert, double* dual_inf_cert) {
    if (int e = need_state(h, "mpcqp_get_certificates")) return e;
    if (!h) return fail(MPCQP_EINVAL, "NULL handle");
    if (h->staged) {
        for (auto& s : h->shards) {
            const Stage g = stage_of(h, s);
            if (prim_inf_cert) std::copy(g.dyc, g.dyc + s.B * h->m, prim_inf_cert + s.b0 * h->m);
            if (dual_inf_cert) std::copy(g.dxc, g.dxc + s.B * h->n, dual_inf_cert + s.b0 * h->n);
        }
        return 0;
    }
    for (auto& s : h->shards) {
        HIPCHK(hipSetDevice(s.dev));
        if (prim_inf_cert)
            HIPCHK(hipMemcpy(prim_inf_cert + s.b0 * h->m, s.kp.dyc, sizeof(double) * s.B * h->m, hipMemcpyDeviceToHost));
        if (dual_inf_cert)
            HIPCHK(hipMemcpy(dual_inf_cert + s.b0 * h->n, s.kp.dxc, sizeof(double) * s.B * h->n, hipMemcpyDeviceToHost));
    }
    return 0;
}

int mpcqp_create(int32_t n, int32_t m, const int32_t* Pp, const int32_t* Pi, const int32_t* Ap,
                 const int32_t* Ai, int64_t B, const mpcqp_settings* settings, int32_t device,
                 mpcqp_handle** out) {
    return make_handle(n, m, Pp, Pi, Ap, Ai, B, settings, std::vector<int>{device}, false, out);
}

static hipStream_t pick(Shard& s, void* stream) { return stream ? (hipStream_t)stream : s.stream; }

// on: the record this launch kind goes to is enabled (collect: solve launches,
// collect_setup: setup launches)
static int ev_begin(bool on, std::vector<std::pair<hipEvent_t, hipEvent_t>>& v, hipStream_t st) {
    if (!on) return 0;
    hipEvent_t a, b;
    HIPCHK(hipEventCreate(&a));
    HIPCHK(hipEventCreate(&b));
    HIPCHK(hipEventRecord(a, st));
    v.push_back({a, b});
    return 0;
}
static int ev_end(bool on, std::vector<std::pair<hipEvent_t, hipEvent_t>>& v, hipStream_t st) {
    if (!on || v.empty()) return 0;
    HIPCHK(hipEventRecord(v.back().second, st));
    return 0;
}

int mpcqp_setup_device(mpcqp_handle* h, const double* dPx, const double* dAx, const double* dq,
                       const double* dl, const double* du, void* stream) {
    if (!h || h->shards.size() != 1) return fail(MPCQP_EINVAL, "device entry points need a single-device handle");
    h->staged = false;  // (device work: the staged results of the last solve are stale)
    Shard& s = h->shards[0];
    hipStream_t st = pick(s, stream);
    HIPCHK(hipSetDevice(s.dev));
    if (int e = stream_enter(s, st)) return e;
    if (h->collect_setup)
        if (int e = ev_begin(h->collect_setup, h->ev_setup, st)) return e;
    HIPCHK(launch_setup(s.kp, s.B, dPx, dAx, dq, dl, du, st));
    if (h->collect_setup)
        if (int e = ev_end(h->collect_setup, h->ev_setup, st)) return e;
    h->state_gone = false;
    return stream_leave(s, st);
}

int mpcqp_update_device(mpcqp_handle* h, const double* dq, const double* dl, const double* du, void* stream) {
    if (int e = need_state(h, "mpcqp_update_device")) return e;
    if (!h || h->shards.size() != 1) return fail(MPCQP_EINVAL, "device entry points need a single-device handle");
    h->staged = false;  // (device work: the staged results of the last solve are stale)
    Shard& s = h->shards[0];
    hipStream_t st = pick(s, stream);
    HIPCHK(hipSetDevice(s.dev));
    if (int e = stream_enter(s, st)) return e;
    HIPCHK(launch_update(s.kp, s.B, dq, dl, du, st));
    return stream_leave(s, st);
}

int mpcqp_warm_start_device(mpcqp_handle* h, const double* dx, const double* dy, void* stream) {
    if (int e = need_state(h, "mpcqp_warm_start_device")) return e;
    if (!h || h->shards.size() != 1) return fail(MPCQP_EINVAL, "device entry points need a single-device handle");
    h->staged = false;  // (device work: the staged results of the last solve are stale)
    Shard& s = h->shards[0];
    hipStream_t st = pick(s, stream);
    HIPCHK(hipSetDevice(s.dev));
    if (int e = stream_enter(s, st)) return e;
    HIPCHK(launch_warm(s.kp, s.B, dx, dy, st));
    s.kp.warm_start = 1;
    h->set.warm_start = 1;
    return stream_leave(s, st);
}

int mpcqp_setup_warm_device(mpcqp_handle* h, const double* dPx, const double* dAx, const double* dq,
                            const double* dl, const double* du, const double* dx0, const double* dy0, void* stream) {
    if (!h || h->shards.size() != 1) return fail(MPCQP_EINVAL, "device entry points need a single-device handle");
    h->staged = false;  // (device work: the staged results of the last solve are stale)
    Shard& s = h->shards[0];
    hipStream_t st = pick(s, stream);
    HIPCHK(hipSetDevice(s.dev));
    if (int e = stream_enter(s, st)) return e;
    if (h->collect_setup)
        if (int e = ev_begin(h->collect_setup, h->ev_setup, st)) return e;
    HIPCHK(launch_setup_warm(s.kp, s.B, dPx, dAx, dq, dl, du, dx0, dy0, st));
    if (h->collect_setup)
        if (int e = ev_end(h->collect_setup, h->ev_setup, st)) return e;
    h->state_gone = false;
    s.kp.warm_start = 1;
    h->set.warm_start = 1;
    return stream_leave(s, st);
}

int mpcqp_setup_warm_fused(const mpcqp_handle* h) {
    if (!h || h->shards.empty()) return fail(MPCQP_EINVAL, "mpcqp_setup_warm_fused: null handle");
    return setup_warm_fused(h->shards[0].kp) ? 1 : 0;
}

int mpcqp_solve_device(mpcqp_handle* h, double* dx, double* dy, int32_t* dstatus, int32_t* diters, void* stream) {
    if (int e = need_state(h, "mpcqp_solve_device")) return e;
    if (!h || h->shards.size() != 1) return fail(MPCQP_EINVAL, "device entry points need a single-device handle");
    h->staged = false;  // (device work: the staged results of the last solve are stale)
    Shard& s = h->shards[0];
    hipStream_t st = pick(s, stream);
    HIPCHK(hipSetDevice(s.dev));
    if (int e = stream_enter(s, st)) return e;
    // an event pair around the launch only while timing is on (mpcqp_setup_solve_device)
    if (h->collect)
        if (int e = ev_begin(h->collect, h->ev_solve, st)) return e;
    KParams k = s.kp;  // the solve kernel writes status / iter into the caller's arrays as well
    k.ostat = dstatus;
    k.oiter = diters;
    HIPCHK(launch_solve(k, s.B, dx, dy, 0, st));
    if (h->collect) {
        if (int e = ev_end(h->collect, h->ev_solve, st)) return e;
        h->last_pair = h->ev_solve.back();
    }
    HIPCHK(launch_order(k, s.B, st));
    h->timed = true;
    return stream_leave(s, st);
}

int mpcqp_setup_solve_device(mpcqp_handle* h, const double* dPx, const double* dAx, const double* dq,
                             const double* dl, const double* du, double* dx, double* dy, int32_t* dstatus,
                             int32_t* diters, void* stream) {
    if (!h || h->shards.size() != 1) return fail(MPCQP_EINVAL, "device entry points need a single-device handle");
    h->staged = false;  // (device work: the staged results of the last solve are stale)
    Shard& s = h->shards[0];
    hipStream_t st = pick(s, stream);
    HIPCHK(hipSetDevice(s.dev));
    if (int e = stream_enter(s, st)) return e;
    // no event between the kernels unless timing is on: every recorded event is a packet
    // the command processor completes between two launches (≈12 us per step measured on
    // the cfg-2 bench, 2.33 -> 2.40 M solves/s without them)
    if (h->collect)
        if (int e = ev_begin(h->collect, h->ev_solve, st)) return e;
    KParams k = s.kp;
    k.ostat = dstatus;
    k.oiter = diters;
    const bool one = h->one_shot && one_shot_form(k) > 0;
    HIPCHK(launch_setup_solve(k, s.B, dPx, dAx, dq, dl, du, dx, dy, st, one));
    h->state_gone = one;
    if (h->collect) {
        if (int e = ev_end(h->collect, h->ev_solve, st)) return e;
        h->last_pair = h->ev_solve.back();
    }
    HIPCHK(launch_order(k, s.B, st));
    h->timed = true;
    return stream_leave(s, st);
}

void* mpcqp_get_stream(const mpcqp_handle* h) {
    return (h && !h->shards.empty()) ? (void*)h->shards[0].stream : nullptr;
}

int mpcqp_set_one_shot(mpcqp_handle* h, int32_t on) {
    if (!h || h->shards.size() != 1) return fail(MPCQP_EINVAL, "device entry points need a single-device handle");
    h->one_shot = on != 0;
    return 0;
}

int mpcqp_one_shot_applies(const mpcqp_handle* h) {
    return (h && h->shards.size() == 1) ? one_shot_form(h->shards[0].kp) : 0;
}

int mpcqp_set_shared_matrices(mpcqp_handle* h, int32_t shared) {
    if (!h || h->shards.size() != 1) return fail(MPCQP_EINVAL, "device entry points need a single-device handle");
    h->staged = false;  // (device work: the staged results of the last solve are stale)
    h->shards[0].kp.mat_shared = shared ? 1 : 0;
    return 0;
}

int mpcqp_synchronize(mpcqp_handle* h) {
    if (!h) return fail(MPCQP_EINVAL, "NULL handle");
    return sync_all(h);
}

double mpcqp_last_kernel_ms(mpcqp_handle* h) {
    if (!h || h->shards.size() != 1 || !h->last_pair.first) return -1.0;
    Shard& s = h->shards[0];
    float ms = 0.f;
    if (hipSetDevice(s.dev) != hipSuccess) return -1.0;
    if (hipEventSynchronize(h->last_pair.second) != hipSuccess) return -1.0;
    if (hipEventElapsedTime(&ms, h->last_pair.first, h->last_pair.second) != hipSuccess) return -1.0;
    return ms;
}

static int drain(std::vector<std::pair<hipEvent_t, hipEvent_t>>& v, double* total) {
    double t = 0.0;
    for (auto& e : v) {
        float ms = 0.f;
        HIPCHK(hipEventSynchronize(e.second));
        HIPCHK(hipEventElapsedTime(&ms, e.first, e.second));
        t += ms;
        (void)hipEventDestroy(e.first);
        (void)hipEventDestroy(e.second);
    }
    if (total) *total = t;
    v.clear();
    return 0;
}

int mpcqp_timing(mpcqp_handle* h, int32_t enable) {
    if (!h || h->shards.size() != 1) return fail(MPCQP_EINVAL, "timing needs a single-device handle");
    if (int e = hipSetDevice(h->shards[0].dev) == hipSuccess ? 0 : fail(MPCQP_EDEVICE, "hipSetDevice")) return e;
    double t;
    if (int e = drain(h->ev_setup, &t)) return e;
    if (int e = drain(h->ev_solve, &t)) return e;
    h->last_pair = {nullptr, nullptr};  // the drained events are gone
    h->collect = (enable & 1) != 0;
    h->collect_setup = (enable & 2) != 0;
    return 0;
}

int mpcqp_timing_read(mpcqp_handle* h, double* setup_ms, int32_t* n_setup, double* solve_ms, int32_t* n_solve) {
    if (!h || h->shards.size() != 1) return fail(MPCQP_EINVAL, "timing needs a single-device handle");
    HIPCHK(hipSetDevice(h->shards[0].dev));
    if (n_setup) *n_setup = (int32_t)h->ev_setup.size();
    if (n_solve) *n_solve = (int32_t)h->ev_solve.size();
    if (int e = drain(h->ev_setup, setup_ms)) return e;
    if (int e = drain(h->ev_solve, solve_ms)) return e;
    h->last_pair = {nullptr, nullptr};
    return 0;
}

int mpcqp_get_plan_info(const mpcqp_handle* h, mpcqp_plan_info* info) {
    if (!h || !info) return fail(MPCQP_EINVAL, "NULL argument");
    info->n = h->n; info->m = h->m; info->nb = h->plan->nb; info->block = kS;
    info->npad = h->plan->npad; info->max_level = h->plan->max_level;
    info->batch = h->B; info->n_devices = (int)h->shards.size();
    info->lds_bytes_solve = h->shards.empty() ? 0 : (int64_t)lds_kernel_bytes(h->shards[0].kp);
    info->bytes_per_instance = (int64_t)(workspace_bytes(*h->plan, 1, false));
    info->amax = h->plan->amax;
    info->gather_k = h->plan->gather_k;
    info->variant = h->shards.empty() ? -1 : h->shards[0].kp.variant;
    info->threads_per_qp = h->shards.empty() ? 0 : solve_threads(h->shards[0].kp.variant);
    info->n_eliminated = h->plan->ne;
    info->plan_choice = h->plan->choice;
    return 0;
}

int mpcqp_plan_preview(int32_t n, int32_t m, const int32_t* Pp, const int32_t* Pi, const int32_t* Ap,
                       const int32_t* Ai, const mpcqp_settings* settings, mpcqp_plan_info* info, char* note,
                       int32_t note_cap) {
    if (!info || !Pp || !Pi || !Ap || !Ai) return fail(MPCQP_EINVAL, "NULL argument");
    mpcqp_settings st;
    if (settings) st = *settings;
    else mpcqp_default_settings(&st);
    if (int e = validate_settings(st)) return e;
    Plan pl;
    std::string err = choose_plan(n, m, Pp, Pi, Ap, Ai, st, pl);
    if (note && note_cap > 0) snprintf(note, (size_t)note_cap, "%s", pl.choice_note.c_str());
    if (!err.empty()) return fail(err.rfind("unsupported", 0) == 0 ? MPCQP_EUNSUPPORTED : MPCQP_EINVAL, "%s", err.c_str());
    KParams k{};
    shape_params(pl, k);
    k.variant = solve_variant(k);
    if (const char* ev = getenv("MPCQP_VARIANT"); ev && *ev) {  // the override alloc_shard applies
        const int v = atoi(ev);
        if (!variant_fits(k, v)) return fail(MPCQP_EUNSUPPORTED, "MPCQP_VARIANT=%d does not fit this plan", v);
        k.variant = v;
    }
    k.mode = k.variant >= 0 ? solve_mode(k.variant) : 0;
    *info = mpcqp_plan_info{};
    info->n = n; info->m = m; info->nb = pl.nb; info->block = kS; info->npad = pl.npad;
    info->max_level = pl.max_level;
    info->lds_bytes_solve = k.variant >= 0 ? (int64_t)lds_kernel_bytes(k) : 0;
    info->bytes_per_instance = (int64_t)workspace_bytes(pl, 1, false);
    info->amax = pl.amax; info->gather_k = pl.gather_k; info->variant = k.variant;
    info->threads_per_qp = k.variant >= 0 ? solve_threads(k.variant) : 0;
    info->n_eliminated = pl.ne; info->plan_choice = pl.choice;
    return 0;
}

int mpcqp_debug_phase_times(mpcqp_handle* h, int64_t* out) {
    if (!h || !out) return fail(MPCQP_EINVAL, "NULL argument");
    for (auto& s : h->shards)
        if (!s.kp.prof) return fail(MPCQP_EINVAL, "phase timers not enabled (set MPCQP_PHASE_PROF=1 before create)");
    if (int e = sync_all(h)) return e;
    for (auto& s : h->shards) {
        HIPCHK(hipSetDevice(s.dev));
        HIPCHK(hipMemcpy(out + s.b0 * kProfSlots, s.kp.prof, sizeof(int64_t) * s.B * kProfSlots, hipMemcpyDeviceToHost));
    }
    return 0;
}

int mpcqp_debug_dispatch_order(mpcqp_handle* h, int32_t* out) {
    if (!h || !out) return fail(MPCQP_EINVAL, "NULL argument");
    if (int e = sync_all(h)) return e;
    for (auto& s : h->shards) {
        int32_t* o = out + s.b0;
        if (!s.kp.order) {
            for (long i = 0; i < s.B; ++i) o[i] = (int32_t)(s.b0 + i);
            continue;
        }
        HIPCHK(hipSetDevice(s.dev));
        HIPCHK(hipMemcpy(o, s.kp.order, sizeof(int32_t) * s.B, hipMemcpyDeviceToHost));
        for (long i = 0; i < s.B; ++i) o[i] += (int32_t)s.b0;
    }
    return 0;
}

int mpcqp_debug_copy(const double* src, double* dst, int64_t n, int32_t reps, void* stream, double* ms) {
    if (!src || !dst || !ms || n <= 0 || n % 16384 || reps <= 0 || ((uintptr_t)src | (uintptr_t)dst) & 15)
        return fail(MPCQP_EINVAL, "mpcqp_debug_copy: n > 0, n %% 16384 == 0, reps > 0, 16-byte aligned buffers");
    hipStream_t st = (hipStream_t)stream;
    if (st) {  // the events and kernels on the device the caller's stream belongs to
        int dev = 0;
        HIPCHK(hipStreamGetDevice(st, &dev));
        HIPCHK(hipSetDevice(dev));
    }
    struct Events {  // destroyed on every return path (HIPCHK returns early)
        hipEvent_t a = nullptr, b = nullptr;
        ~Events() {
            if (a) (void)hipEventDestroy(a);
            if (b) (void)hipEventDestroy(b);
        }
    } ev;
    HIPCHK(hipEventCreate(&ev.a));
    HIPCHK(hipEventCreate(&ev.b));
    hipEvent_t a = ev.a, b = ev.b;
    double best = 0.0;
    for (int form = 0; form < 5; ++form) {  // the fastest of the five forms (kernels.hip::launch_copy16)
        HIPCHK(launch_copy16(src, dst, n, st, form));  // (warm-up)
        HIPCHK(hipEventRecord(a, st));
        for (int r = 0; r < reps; ++r) HIPCHK(launch_copy16(src, dst, n, st, form));
        HIPCHK(hipEventRecord(b, st));
        HIPCHK(hipEventSynchronize(b));
        float t = 0.0f;
        HIPCHK(hipEventElapsedTime(&t, a, b));
        const double per = (double)t / reps;
        if (form == 0 || per < best) best = per;
    }
    *ms = best;
    return 0;
}

void mpcqp_free(mpcqp_handle* h) {
    if (!h) return;
    if (!h->shards.empty() && hipSetDevice(h->shards[0].dev) == hipSuccess) {
        double t;
        drain(h->ev_setup, &t);
        drain(h->ev_solve, &t);
    }
    for (auto& s : h->shards) free_shard(s);
    delete h;
}

}  // extern "C"
