// kernels.h -- device-side interface shared by kernels.hip and api.hip.
#pragma once
#include <hip/hip_runtime.h>

#include "plan.h"

namespace mpcqp {

constexpr int kThreads = 256;
constexpr int kThreadsBig = 512;  // solve_big.hip (long horizons)
constexpr int kDenseR = 104;      // solve_dense.hip: register row length of M^{-1} (variables per QP)
constexpr int kProfSlots = 24;  // factor, rhs, bt_solve, update, checks, tail, total cycles, total 100 MHz ticks,
                                // factor split: assembly, F/S products, Gauss-Jordan, block epilogue,
                                // solve split (wave kernels): phase A, phase B, phase C, spare,
                                // 16-23: per-wave sub-phase times (solve_big.hip's interface form: the
                                // chain waves' own forward / backward times, wave 0's T and X)

// status values (OSQP constants.h)
enum : int {
    MPCQP_DUAL_INFEASIBLE_INACCURATE_ = 4,
    MPCQP_PRIMAL_INFEASIBLE_INACCURATE_ = 3,
    MPCQP_SOLVED_INACCURATE_ = 2,
    MPCQP_SOLVED_ = 1,
    MPCQP_MAX_ITER_REACHED_ = -2,
    MPCQP_PRIMAL_INFEASIBLE_ = -3,
    MPCQP_DUAL_INFEASIBLE_ = -4,
    MPCQP_NON_CVX_ = -7,
    MPCQP_UNSOLVED_ = -10,
};

// Everything a kernel needs: plan (shared pattern, read-only) + per-instance
// workspace (instance-major arrays) + settings.  Passed by value.
struct KParams {
    int n, m, nb, npad, nnzP, nnzA, amax, gk, pk, ntgt, term_max;
    int gk1;          // most nonzeros in a row >= 128 (the two-wave kernel's second row slot)
    int gkr, gkc;     // most nonzeros in a row / a column of A (gk = the larger)
    int bmax, pmeet;  // two-sided factorisation (solve_big.hip): tail width, meeting block
    int ifok;         // the interface form of the two-sided solve fits (solve_big.hip::iface_solve):
                      // amax, bmax <= 16 and the meeting block's top rows and window disjoint
    int bsz01, bsz23; // largest of blocks 0 and 1 / 2 and 3 (real columns; nb = 4 plans)
    int variant;  // solve-kernel instantiation (solve.hip: launch_solve)
    int mode;     // factor storage of that variant (solve.hip: factorize)
    // plan
    const int *pad_var, *acsc_ptr, *acsc_row, *acsc_v, *acsr_ptr, *acsr_col, *acsr_v;
    const int *psym_ptr, *psym_col, *psym_v, *p_r, *p_c, *a_r, *a_c;
    const int *asm_blk_ptr, *asm_tgt, *tterm, *acsr_pos, *gcol, *grow, *gpsym, *toff;
    const int* bsize;  // [nb] real variables of each block (the rest of its 32 are padding, at the end)
    const int* tcnt;   // [ntgt] assembly terms per target, descending within a block (plan.cpp)
    // eliminated variables (plan.h, Plan::eown): padded columns [nb S, nb S + ne), owned by
    // block column eown[pc]'s lane; etterm: the ELL terms of their K_jj / K_pj (target 2e / 2e + 1)
    int ne, ecnt, eterm_max;
    const int *eown, *etterm;
    // workspace
    double *Px, *Ax, *q, *D, *l, *u, *E, *x, *z, *y, *scal, *F, *H, *Si, *dyc, *dxc;
    double* Kd;  // dense-inverse rows of the four-wave kernel's DK form (dense_rows_doubles per instance), or null
    double *obj, *pri, *dua, *rho_est;
    signed char* ct;
    int *status, *iter, *rho_upd, *err;
    // per instance: 1 while the workspace factor (F / H / Si: the long-horizon kernel, mode 3)
    // is the one of the current data, rho and row classes, so that k_solve_b's next solve starts
    // without refactoring (a setup's convexity check, a previous solve).  Cleared by every setup,
    // by an update that moves a row's class, by a rho set through update_settings and by polish
    int* ffresh;
    int reuse;  // k_solve_b may start from a fresh workspace factor (MPCQP_FACTOR_REUSE=0: never, A/B)
    int apart;  // k_solve_b's bottom chain may update the middle block in place (solve_big.hip::middle_apart;
                // MPCQP_MIDDLE_APART=0: never, A/B)
    int *ostat, *oiter;  // per-call copies of status / iter (mpcqp_solve_device's outputs), or null
    const struct KParams* self;  // device copy of this block (read by the out-of-line device functions)
    long long* prof;  // optional per-instance phase timers (MPCQP_PHASE_PROF=1), kProfSlots each
    // settings
    double sigma, alpha, eps_abs, eps_rel, eps_pinf, eps_dinf, rho0, rho_tol, delta;
    int max_iter, scaling, check_term, warm_start, adaptive_rho, rho_interval, scaled_term;
    int polish, refine_iter;
    int* pstat;  // per instance: 0 polish not run, 1 polished solution taken, -1 rejected
    // dispatch order of the solve kernels: workgroup slot -> instance, or null (identity).
    // Rewritten after every solve by launch_order (longest previous solve first).
    const int* order;
    long slots;  // workgroups of the solve kernel resident at once on the device (CUs x occupancy)
    // the four- and two-wave kernels (k_solve_w4 / k_setup_solve_w4, k_solve_w2 /
    // k_setup_solve_w2) sort the order themselves in their last workgroup (device_common.h::order_epilogue)
    // when the batch is at most kOrderFuseMax: arrival counter (zero between launches), or null
    int* done;
    // setup calls: P and A values shared by every instance (Px[nnzP], Ax[nnzA] instead of
    // B copies; LTI MPC -- mpcqp_set_shared_matrices)
    int mat_shared;
    // k_solve_b's factorisation chain runs on LDS copies of its tiles (solve_big.hip::
    // factorize2s_lds_chain; MPCQP_LDS_CHAIN=0: the workspace form, A/B)
    int lchain;
    // dispatch prediction with history (kernels.hip::k_order): key = max(iter, pred), then
    // pred = key * odecay / 8 per instance -- an instance that was slow in a recent solve keeps
    // an early slot for a few solves (MPCQP_ORDER_DECAY=0..8, default 7; 0: the previous count
    // alone)
    int* pred;
    int odecay;
    // k_solve_b's persistent form (solve_big.hip; MPCQP_PERSIST=0: off): queue[0] the next index
    // of the order, queue[1] the workgroups done (zero between launches); persist / qn per launch
    int* queue;
    int qpersist;
    int persist;
    long qn;
    // the wide batch setup's plan lists (plan.h wide_*, csc_pos)
    const int *wcg, *wpg, *wrg, *was, *wps, *csc_pos;
};
constexpr long kOrderFuseMax = 16384;  // larger batches sort in k_order (1024 threads)

size_t lds_setup_bytes(const KParams& p);
size_t lds_solve_bytes(const KParams& p);
size_t lds_solve_bytes_big(const KParams& p);  // + the F rows of solve_big.hip
size_t lds_kernel_bytes(const KParams& p);     // what the chosen variant's kernel allocates
// error text for mpcqp_last_error() (api.hip); returns code
int set_error(int code, const char* fmt, ...);

// keep: the rescaling of a matrix update (launch_update_mat) -- x, z, y, the row classes
// and rho are left as they are
hipError_t launch_setup(const KParams& p, long B, const double* Px, const double* Ax, const double* q,
                        const double* l, const double* u, hipStream_t st, bool keep = false);
// osqp_update_P_A: unscale the workspace's data into the *_io setup inputs (user order),
// write the new values (B x nP / B x nA, at the given indices or all), scale afresh
hipError_t launch_update_mat(const KParams& p, long B, double* Px_io, double* Ax_io, double* q_io, double* l_io,
                             double* u_io, const double* Px_new, const int* Px_idx, int nP, const double* Ax_new,
                             const int* Ax_idx, int nA, hipStream_t st);
hipError_t launch_update(const KParams& p, long B, const double* q, const double* l, const double* u,
                         hipStream_t st);
hipError_t launch_warm(const KParams& p, long B, const double* x, const double* y, hipStream_t st);
// launch_setup then launch_warm(x0, y0), identical results; one kernel where the wide batch
// setup applies (setup_warm_fused: the long-horizon plans, setup_wide.h WARM)
bool setup_warm_fused(const KParams& p);
hipError_t launch_setup_warm(const KParams& p, long B, const double* Px, const double* Ax, const double* q,
                             const double* l, const double* u, const double* x0, const double* y0, hipStream_t st);
// longest-processing-time dispatch: sort the instances by the iteration count of the
// solve just run (descending) into p.order, for the next solve on this workspace
hipError_t launch_order(const KParams& p, long B, hipStream_t st);
// order[i] = i (the identity dispatch order of a fresh workspace), enqueued on st
hipError_t launch_iota(int* order, long B, hipStream_t st);
// Small host calls' result staging (api.hip::mpcqp_solve_batch): every array a solve returns
// gathered into one device buffer by one kernel, so that one copy brings it to pinned memory
// (eleven D2H copies ran as eleven ~5 us blit kernels one after another)
struct GatherSeg {
    const void* src;  // nullptr: fill with zeros
    long off;         // byte offset in the destination
    long cnt;         // elements
    int sz;           // element bytes: 8 or 4
};
constexpr int kGatherMax = 12;
struct GatherList {
    GatherSeg seg[kGatherMax];
    int nseg;
    long most;  // the largest cnt
};
hipError_t launch_gather(const GatherList& g, void* dst, hipStream_t st);
// streaming device copy of n doubles (n % 16384 == 0) in one of three forms (kernels.hip),
// mpcqp_debug_copy
hipError_t launch_copy16(const double* src, double* dst, long n, hipStream_t st, int form);
// doubles per instance of the four-wave kernel's dense-inverse rows (KParams::Kd): 256 lanes x
// (NB0 + NB1 = 54) for plans of four blocks without eliminated columns (solve_wave.hip, DK).
// The DK form was measured and not taken: it is compiled into the experimental
// builds only and runs there under MPCQP_DENSE_W4=1; dense_w4_on() is false in the production
// library, so no workspace is carved for it there (cfg 2: 231 -> 121 kB per instance).
constexpr long kDenseRowDoubles = 256L * 54;
bool dense_w4_on();  // solve_wave.hip: experimental build and MPCQP_DENSE_W4=1
inline long dense_rows_doubles(int nb, int ne) { return nb == 4 && ne == 0 && dense_w4_on() ? kDenseRowDoubles : 0; }
int solve_variant(const KParams& p);  // -1: no instantiation fits the plan
int solve_mode(int variant);
int solve_threads(int variant);  // workgroup size of the variant's kernel
bool variant_fits(const KParams& p, int variant);
hipError_t launch_solve(const KParams& p, long B, double* xo, double* yo, int factor_only, hipStream_t st);
// setup + solve of the same inputs (solve_wave.hip): one fused kernel where the variant
// allows it, else launch_setup then launch_solve
hipError_t launch_setup_solve(const KParams& p, long B, const double* Px, const double* Ax, const double* q,
                              const double* l, const double* u, double* xo, double* yo, hipStream_t st,
                              bool one_shot = false);
// the one-shot fused kernel's form for the plan (solve_wave.hip): 0 none (not the fused four-wave
// kernel, or polish), 1 the G blocks in the workspace, 2 the G blocks in an LDS region of their
// own (two workgroups per CU still fit), 3 the G blocks straight into the solve's LDS copy
// (factorize_w4_gl); *lds = its dynamic LDS bytes
int one_shot_form(const KParams& p, size_t* lds = nullptr);
// What a solve launch runs: the variant's kernel, workgroup size and dynamic LDS.  The
// launch_solve_* functions given a non-null ref only fill it in (no launch).
struct KernelRef {
    const void* fn;
    int threads;
    size_t lds;
};
// resident workgroups of the variant's kernel per CU (hipOccupancyMaxActiveBlocksPerMultiprocessor)
int solve_blocks_per_cu(const KParams& p);
// dense-inverse kernel (solve_dense.hip), variant 16, and its LDS bytes
hipError_t launch_solve_dense(const KParams& p, long B, double* xo, double* yo, int factor_only, hipStream_t st,
                        KernelRef* ref = nullptr);
size_t lds_dense_bytes(const KParams& p);
size_t lds_w2_bytes(const KParams& p);  // solve_wave.hip, variant 10
// solution polishing (OSQP 0.6 polish.c) after the solve; launch_solve runs it when p.polish
hipError_t launch_polish(const KParams& p, long B, double* xo, double* yo, hipStream_t st);
// one-wave-per-QP kernel (solve_wave.hip), variants 8 and 9
hipError_t launch_solve_wave(const KParams& p, long B, double* xo, double* yo, int factor_only, hipStream_t st,
                        KernelRef* ref = nullptr);
// one 512-thread workgroup per QP, alone on its CU, the dense-inverse solve held in registers
// (solve_heavy.hip, variant 19): the latency form for a batch's predicted-slowest instances
bool heavy_fits(const KParams& p);
size_t heavy_lds(const KParams& p);
hipError_t launch_solve_heavy(const KParams& p, long B, double* xo, double* yo, int factor_only, hipStream_t st,
                              KernelRef* ref = nullptr);
hipError_t launch_setup_solve_heavy(const KParams& p, long B, const double* Px, const double* Ax, const double* q,
                                    const double* l, const double* u, double* xo, double* yo, hipStream_t st);
// 512-thread long-horizon kernel (solve_big.hip), variants 11-13
hipError_t launch_solve_big(const KParams& p, long B, double* xo, double* yo, int factor_only, hipStream_t st,
                        KernelRef* ref = nullptr);

}  // namespace mpcqp
