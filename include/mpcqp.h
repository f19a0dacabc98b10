/*
 * mpcqp.h -- C ABI of the MI355X batched linear-MPC QP solver (libmpcqp.so).
 *
 * Drop-in boundary for the reference's `osqp.OSQP()` call sites.  Each entry
 * point below replaces one step of the reference's OSQP usage:
 *
 *   mpcqp_setup_batch     <- prob = osqp.OSQP(); prob.setup(P, q, A, l, u, **settings)
 *                            vehicle_lateral_mpc_slack_increment.py:118,121
 *                            Control/MPC/mpc_kinematics.py:194-195
 *                            Control/MPC/mpc_dynamics.py:240-241,392-393
 *                            Control/MPC/mpc_kinematics_pred_matrix.py:195-196,260-261,346-347
 *                            Control/MPC/mpc_increment_kinematics_pred_matrix.py:241-242
 *                            Control/MPC/mpc_bottleneck_check.py:197-198
 *                            Control/MPC/mpc_incre_kine_func.py:179-180
 *   mpcqp_update_batch    <- prob.update(q=q_new, l=l_new, u=u_new)
 *                            vehicle_lateral_mpc_slack_increment.py:237,269
 *   mpcqp_update_settings <- prob.update_settings(**kwargs)   (osqp API; not called by the reference)
 *   mpcqp_update_matrices_batch <- prob.update(Px=, Px_idx=, Ax=, Ax_idx=)
 *                            vehicle_lateral_mpc_slack_increment.py:236 (commented out there)
 *   mpcqp_warm_start_batch<- prob.warm_start(x=..., y=...)   (osqp API; used for
 *                            the receding-horizon shift)
 *   mpcqp_solve_batch     <- res = prob.solve(); res.x, res.y, res.info.status, res.info.iter
 *                            vehicle_lateral_mpc_slack_increment.py:248,252,256
 *                            Control/MPC/mpc_dynamics.py:396,406-407
 *   mpcqp_free            <- end of the OSQP object's lifetime
 *
 * One handle holds B independent QP instances that SHARE one sparsity pattern
 * (P upper-triangular CSC n x n, A CSC m x n, int32, 0-based) and carry their
 * own values.  Per-instance arrays are instance-major:  Px[B*nnzP], Ax[B*nnzA],
 * q[B*n], l[B*m], u[B*m], x[B*n], y[B*m].  Values follow the order of the
 * pattern's data arrays (osqp-python keeps triu(P) in CSC order).
 *
 * Ownership: every input is copied into device memory during the call; the
 * caller may free or reuse its buffers afterwards.  Outputs go to
 * caller-allocated buffers.  Host-pointer entry points block until results
 * are on the host; *_device entry points take device pointers on the
 * handle's (single) device and enqueue on `stream` (hipStream_t, NULL = the
 * handle's own stream) without synchronising.  Calls on one handle are
 * stream-ordered by the library: they share the handle's workspace, including
 * the dispatch order each solve rewrites for the next one (longest previous
 * solve first; setting MPCQP_DISPATCH=identity before mpcqp_create /
 * mpcqp_setup_batch turns it off), so a call enqueued on a different stream
 * than the previous call on the handle first waits (hipStreamWaitEvent) for
 * that call's work.  The caller still orders its own buffers (inputs written
 * on another stream, outputs read elsewhere).  The order moves instances
 * between workgroups, never their results.
 *
 * Errors: entry points return 0 on success or an MPCQP_E* code; the message
 * is in mpcqp_last_error() (thread-local).  Numerical outcomes never fail a
 * call: they are reported per instance in status[] with OSQP's values.
 * A handle must be used from one host thread at a time.
 */
#ifndef MPCQP_H
#define MPCQP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* per-instance status (same values as OSQP's constants.h) */
#define MPCQP_DUAL_INFEASIBLE_INACCURATE 4
#define MPCQP_PRIMAL_INFEASIBLE_INACCURATE 3
#define MPCQP_SOLVED_INACCURATE 2
#define MPCQP_SOLVED 1
#define MPCQP_MAX_ITER_REACHED (-2)
#define MPCQP_PRIMAL_INFEASIBLE (-3)
#define MPCQP_DUAL_INFEASIBLE (-4)
#define MPCQP_NON_CVX (-7)
#define MPCQP_UNSOLVED (-10)

/* call error codes */
#define MPCQP_OK 0
#define MPCQP_EINVAL 1        /* bad argument / data validation (e.g. l > u) */
#define MPCQP_EUNSUPPORTED 2  /* sparsity structure or setting not supported */
#define MPCQP_EDEVICE 3       /* HIP runtime error / no device */
#define MPCQP_ENOMEM 4
#define MPCQP_ENONCVX 5       /* mpcqp_setup_batch: an instance's P is not convex (OSQP_NONCVX_ERROR) */

typedef struct {
    double rho, sigma, alpha;
    double eps_abs, eps_rel, eps_prim_inf, eps_dual_inf;
    double adaptive_rho_tolerance;
    int32_t max_iter, scaling, check_termination, warm_start;
    int32_t adaptive_rho, adaptive_rho_interval, scaled_termination, polish, verbose;
    double delta;                 /* polish regularisation (OSQP default 1e-6) */
    int32_t polish_refine_iter;   /* polish iterative-refinement steps (OSQP default 3) */
} mpcqp_settings;

typedef struct {
    int32_t n, m, nb, block, npad, max_level;
    int64_t batch;
    int32_t n_devices;
    int64_t lds_bytes_solve;    /* dynamic LDS per workgroup of the ADMM kernel */
    int64_t bytes_per_instance; /* device workspace per instance */
    int32_t amax;               /* coupling rows of the off-diagonal blocks */
    int32_t gather_k;           /* max nonzeros per row / column of A */
    int32_t variant;            /* solve-kernel instantiation in use */
    int32_t threads_per_qp;     /* workgroup size of that kernel */
    int32_t n_eliminated;       /* variables taken out of the block system by a scalar Schur
                                   complement (degree <= 1 vertices of K: slack columns) */
    int32_t plan_choice;        /* 0 plain plan (elimination not tried: polish, MPCQP_ELIM=0, a
                                   variant override), 1 eliminated plan, 2 an eliminated plan was
                                   built but did not fit the four-wave kernel (the reason:
                                   mpcqp_plan_preview's note; MPCQP_PLAN_LOG=1 prints it),
                                   3 nothing to eliminate */
} mpcqp_plan_info;

typedef struct mpcqp_handle mpcqp_handle;

/* OSQP 0.6 defaults; adaptive_rho_interval = 0 resolves to 4*check_termination
 * (OSQP's non-profiling rule, pinned). */
void mpcqp_default_settings(mpcqp_settings *s);

/* Symbolic analysis + allocation + per-instance setup (scaling, rho classes).
 * device_mask: bit d selects HIP device d; 0 = device 0.  The batch is split
 * into contiguous shards across the selected devices (no collectives): every
 * shard's kernels are enqueued (one stream per shard) before the host gathers
 * the results, so the devices run concurrently.  MPCQP_SPLIT=k in the
 * environment (diagnostic) cuts k shards per selected device. */
int mpcqp_setup_batch(int32_t n, int32_t m,
                      const int32_t *Pp, const int32_t *Pi,
                      const int32_t *Ap, const int32_t *Ai,
                      int64_t B, const double *Px, const double *Ax,
                      const double *q, const double *l, const double *u,
                      const mpcqp_settings *settings, uint32_t device_mask,
                      mpcqp_handle **out);

/* (mpcqp_setup_batch, as osqp_setup) returns MPCQP_ENONCVX when an instance's KKT matrix is
 * not quasi-definite (P + sigma I + A' diag(rho) A not positive definite): one factor-only
 * launch of the solve kernel checks every instance.  The device entry points do not check;
 * their solve reports such an instance as non-convex (status -7). */
/* q, l, u may each be NULL (not updated). */
int mpcqp_update_batch(mpcqp_handle *h, const double *q, const double *l, const double *u);
/* osqp_update_P / osqp_update_A / osqp_update_P_A (OSQP 0.6): new values of P's upper
 * triangle and / or A for every instance -- Px is B x nPx, Ax is B x nAx, row-major; each
 * row holds the values at the indices Px_idx / Ax_idx (into the value arrays given to
 * mpcqp_setup_batch, in its CSC order; a repeated index takes its last value), or all
 * nnzP / nnzA values when the index array is NULL (n* then ignored).  Either matrix may be
 * NULL.  As OSQP: the data is unscaled, updated, scaled afresh and refactored at the next
 * solve; x, z, y, rho and the row classes are kept (the iterates stay in the previous
 * scaling).  The sparsity pattern is fixed.  Handles of mpcqp_setup_batch only, not in
 * shared-matrix mode.  MPCQP_ENONCVX when the new matrices are not convex (OSQP's update
 * refactors at once).  Replaces prob.update(Px=, Px_idx=, Ax=, Ax_idx=), which the reference
 * mentions at vehicle_lateral_mpc_slack_increment.py:236 (commented out). */
int mpcqp_update_matrices_batch(mpcqp_handle *h, const double *Px, const int32_t *Px_idx, int32_t nPx,
                                const double *Ax, const int32_t *Ax_idx, int32_t nAx);
/* x, y may each be NULL (keeps the current iterate of that part). */
int mpcqp_warm_start_batch(mpcqp_handle *h, const double *x, const double *y);
/* osqp_update_settings / osqp_update_rho (OSQP 0.6; osqp-python's update_settings): max_iter,
 * eps_abs, eps_rel, eps_prim_inf, eps_dual_inf, rho (with set_rho != 0 only, as osqp-python
 * calls update_rho only when rho is passed: clipped to [1e-6, 1e6], every instance, refactored
 * at the next solve; else each instance keeps the rho its solves adapted to), alpha, delta, polish, polish_refine_iter, scaled_termination,
 * check_termination, warm_start take the new values; sigma, scaling and the adaptive-rho
 * settings must be unchanged (MPCQP_EINVAL otherwise), as OSQP fixes them at setup.  Any
 * handle.  polish = 1 on a handle whose plan eliminated variables (the slack layouts set up
 * without polish) moves the handle onto the plain plan first (polish factors all of K): its
 * data, scaling, iterates, rho and row classes are kept, so the next solve continues exactly
 * as on a handle set up with polish on. */
int mpcqp_update_settings(mpcqp_handle *h, const mpcqp_settings *s, int32_t set_rho);
/* any output may be NULL */
int mpcqp_solve_batch(mpcqp_handle *h, double *x, double *y, int32_t *status, int32_t *iters);
/* info of the last solve; any output may be NULL */
int mpcqp_get_info_batch(mpcqp_handle *h, double *obj_val, double *pri_res, double *dua_res,
                         double *rho_estimate, int32_t *rho_updates);
/* infeasibility certificates of the last solve (OSQP res.prim_inf_cert / dua_inf_cert) */
/* res.info.status_polish per instance (osqp polish.c, run after the solve when
 * settings.polish): 0 not run (status not "solved" or polish off), 1 the polished
 * solution was taken (x, y, obj_val, pri_res, dua_res are the polished ones), -1
 * polishing did not improve the residuals (the ADMM solution stands). */
int mpcqp_get_polish_status(mpcqp_handle *h, int32_t *status_polish);
int mpcqp_get_certificates(mpcqp_handle *h, double *prim_inf_cert, double *dual_inf_cert);

/* ---- device-resident entry points (single-device handles) ---- */
/* Allocate a handle with its workspace but no data (pattern only). */
int mpcqp_create(int32_t n, int32_t m, const int32_t *Pp, const int32_t *Pi,
                 const int32_t *Ap, const int32_t *Ai, int64_t B,
                 const mpcqp_settings *settings, int32_t device, mpcqp_handle **out);
int mpcqp_setup_device(mpcqp_handle *h, const double *dPx, const double *dAx, const double *dq,
                       const double *dl, const double *du, void *stream);
int mpcqp_update_device(mpcqp_handle *h, const double *dq, const double *dl, const double *du,
                        void *stream);
int mpcqp_warm_start_device(mpcqp_handle *h, const double *dx, const double *dy, void *stream);
int mpcqp_solve_device(mpcqp_handle *h, double *dx, double *dy, int32_t *dstatus, int32_t *diters,
                       void *stream);
/* setup + warm start of the same call: mpcqp_setup_device(dPx..du) followed by
 * mpcqp_warm_start_device(dx0, dy0), with identical results (either may be null, as there).
 * Where the wide batch setup applies (the long-horizon plans: setup_wide.h) both run as ONE
 * kernel -- each workgroup scales its instance and forms x = D^-1 x0, y = E^-1 y0 c, z = A x
 * from the values still on chip -- so the warm-start kernel's pass over the workspace goes.
 * The reference's warm-started step prob.setup(...); prob.warm_start(x=, y=); prob.solve()
 * (mpc_dynamics.py:589-610 shifting the previous solution) maps onto it
 * followed by mpcqp_solve_device.  mpcqp_setup_warm_fused: 1 when the handle's plan takes the
 * one-kernel form, 0 when the call runs as the two launches. */
int mpcqp_setup_warm_device(mpcqp_handle *h, const double *dPx, const double *dAx, const double *dq,
                            const double *dl, const double *du, const double *dx0, const double *dy0,
                            void *stream);
int mpcqp_setup_warm_fused(const mpcqp_handle *h);
/* setup + solve of the same inputs in one call: mpcqp_setup_device(dPx..du) followed by
 * mpcqp_solve_device(dx, dy, dstatus, diters), with identical results.  Where the
 * solve kernel allows it -- the four-wave kernel k_setup_solve_w4 (the N=20 lateral
 * layouts: vanilla, and slack once its slack columns are eliminated) or the two-wave
 * kernel k_setup_solve_w2 -- both run as ONE kernel: each workgroup scales its instance
 * and solves it, so no setup kernel and no launch gap stand in front of the slowest
 * instance; the last workgroup also sorts the next dispatch order.  The reference's per-call
 * pattern prob.setup(...); prob.solve() (Control/MPC/mpc_kinematics.py:194-198,
 * mpc_dynamics.py:392-396) maps onto it one-to-one. */
int mpcqp_setup_solve_device(mpcqp_handle *h, const double *dPx, const double *dAx, const double *dq,
                             const double *dl, const double *du, double *dx, double *dy, int32_t *dstatus,
                             int32_t *diters, void *stream);
/* LTI batches ("LTI shared-matrix mode"): with shared != 0 the following
 * mpcqp_setup_device / mpcqp_setup_solve_device calls read ONE Px[nnzP] and ONE Ax[nnzA]
 * for every instance of the batch instead of B copies (the lateral MPC's P and A do not
 * change between instances or steps: vehicle_lateral_mpc_slack_increment.py:79-115). */
int mpcqp_set_shared_matrices(mpcqp_handle *h, int32_t shared);
/* One-shot mode of mpcqp_setup_solve_device (the Control/MPC call pattern: a fresh OSQP()
 * + setup() + solve() every call, mpc_kinematics.py:194-198, so nothing reads the workspace
 * later): while on, the fused setup + solve kernel leaves the scaled problem on chip for the
 * solve instead of in the workspace, stores no warm-start iterates or certificates and keeps the
 * factorisation's G blocks on chip too where the plan leaves room (cfg 2, cfg 3) --
 * the outputs (x, y, status, iters) and the info are the same, bit for bit.  After such a call
 * the calls that read the workspace (update / warm_start / solve, the host batch calls, matrix
 * updates, certificates) fail with MPCQP_EINVAL until a setup.  mpcqp_one_shot_applies: 0 the
 * handle's kernel has no one-shot form (not the fused four-wave kernel, or polish: the call runs
 * as usual), 1 the form with the G blocks in the workspace, 2 with the G blocks in an LDS region
 * of their own, 3 with the G blocks written straight into the solve's LDS copy.  The osqp API
 * never turns it on. */
int mpcqp_set_one_shot(mpcqp_handle *h, int32_t on);
int mpcqp_one_shot_applies(const mpcqp_handle *h);
/* The handle's own hipStream_t (the one a NULL `stream` selects; first shard), so that a
 * caller's kernels (e.g. mpcqp_affine_apply_device) can be ordered with the handle's calls. */
void *mpcqp_get_stream(const mpcqp_handle *h);
/* Blocks until every call enqueued on the handle so far has finished, on the handle's
 * own stream(s) and on the caller stream the last *_device call used. */
int mpcqp_synchronize(mpcqp_handle *h);
/* hipEvent-bracketed time of the last solve: milliseconds, or -1 when unavailable.
 * Recorded only while mpcqp_timing is on, by the host-pointer mpcqp_solve_batch and the
 * *_device entry points alike (no event packet between the kernels otherwise). */
double mpcqp_last_kernel_ms(mpcqp_handle *h);

/* Kernel timing for bench.py's roofline: while enabled, every *_device solve
 * (enable bit 0) / setup (bit 1) launch is bracketed by a hipEvent pair on its
 * stream (no host sync).  mpcqp_timing_read() waits for the recorded events,
 * returns the summed kernel milliseconds and launch counts, and clears the
 * record. */
int mpcqp_timing(mpcqp_handle *h, int32_t enable);
int mpcqp_timing_read(mpcqp_handle *h, double *setup_ms, int32_t *n_setup, double *solve_ms,
                      int32_t *n_solve);

int mpcqp_get_plan_info(const mpcqp_handle *h, mpcqp_plan_info *info);
/* Diagnostics: per-instance phase timers of the last solve (24 int64 per instance:
 * factor, rhs, bt_solve, update, checks, tail shader-clock cycles, total cycles,
 * total 100 MHz wall ticks, then the factorisation split: assembly, F/S products,
 * Gauss-Jordan, block epilogue, then the block-solve split of the wave kernels:
 * phase A, B, C, spare, then eight per-wave sub-phase times of the long-horizon kernel).  Only when MPCQP_PHASE_PROF=1 was set at creation. */
int mpcqp_debug_phase_times(mpcqp_handle *h, int64_t *out);
/* Diagnostics: the dispatch order the next solve will use (B int32 instance indices, each
 * shard's own order offset by its first instance): after a solve, that solve's instances by
 * descending iteration bucket (iter >> shift, 256 buckets; order within a bucket is not
 * fixed).  Sorted in the solve kernel's last workgroup (four- and two-wave kernels) or by
 * k_order (MPCQP_ORDER_KERNEL=1 at creation); identity before the first solve and under
 * MPCQP_DISPATCH=identity. */
int mpcqp_debug_dispatch_order(mpcqp_handle *h, int32_t *out);
/* Diagnostics (bench.py's achievable-HBM reference): `reps` device-to-device
 * copies of n doubles (n a multiple of 16384; 16-byte aligned buffers) by a streaming copy
 * kernel -- 16-byte loads and stores, four or eight in flight per lane, 256-thread workgroups;
 * five forms (non-temporal; default policy; default policy with eight per lane; one pass of a
 * workgroup per 16 KiB, default policy or non-temporal) -- on `stream`
 * (hipStream_t, NULL: the null stream of the current device; a non-NULL stream makes its own
 * device the calling thread's current one), timed by an event pair around each form's launches:
 * *ms = the average per copy of the fastest form.  Blocks until done. */
int mpcqp_debug_copy(const double *src, double *dst, int64_t n, int32_t reps, void *stream, double *ms);

void mpcqp_free(mpcqp_handle *h);
const char *mpcqp_last_error(void);

/* Host-only symbolic analysis (no device needed): block-tridiagonal plan of
 * K = P + sigma I + A' diag(rho) A.  var_pad[n] receives each variable's padded
 * index, bsize[*nb] the block sizes (capacity n).  Used by the CPU test-suite. */
int mpcqp_analyze(int32_t n, int32_t m, const int32_t *Pp, const int32_t *Pi,
                  const int32_t *Ap, const int32_t *Ai, int32_t *nb, int32_t *block,
                  int32_t *var_pad, int32_t *bsize);
/* Same, with `eliminate`: the plan a handle uses for the four-wave kernel -- degree <= 1
 * vertices of K's graph (slack columns) taken out of the blocks (padded indices from
 * nb * block on), blocks packed greedily; n_eliminated (may be NULL) receives their count. */
int mpcqp_analyze_ex(int32_t n, int32_t m, const int32_t *Pp, const int32_t *Pi,
                     const int32_t *Ap, const int32_t *Ai, int32_t eliminate, int32_t *nb,
                     int32_t *block, int32_t *var_pad, int32_t *bsize, int32_t *n_eliminated);

/* Host-only (no device needed): the plan and solve-kernel variant a handle created with
 * this pattern and these settings (NULL: defaults) would take -- the shape fields of
 * mpcqp_plan_info (batch, n_devices = 0) -- and, in note[note_cap] (may be NULL), why an
 * eliminated plan was rejected ("" otherwise).  Used by the CPU test-suite to pin the
 * kernel shape of each workload (e.g. the slack layout's reduced system: 4 blocks, amax <= 8). */
int mpcqp_plan_preview(int32_t n, int32_t m, const int32_t *Pp, const int32_t *Pi,
                       const int32_t *Ap, const int32_t *Ai, const mpcqp_settings *settings,
                       mpcqp_plan_info *info, char *note, int32_t note_cap);

/* ======================================================================
 * The MPC data path around the solver, on the device.
 * Replaces the Python work of Control/MPC/mpc_dynamics.py:main between two
 * osqp solves, batched over B vehicles.  Device pointers, enqueued on `stream`.
 * ====================================================================== */

/* Vehicle_Dynamics(...) constructor arguments (Vehicle_Dynamics/vehicle_models.py:27-50) */
typedef struct {
    double m, l_f, l_r, width, length, C_d, A_f, C_roll, dt;
} mpcqp_vehicle;

/* F2 -- Vehicle_Dynamics.get_dynamics_model (vehicle_models.py:52-340), batched.
 * For b < B, k < N: x = dx[b*x_sb + k*x_sk + 0..6) = (X, Y, yaw, vx, vy, r),
 * u = du[b*u_sb + k*u_sk + 0..2) = (steer, accel)  ->  Ad[(b*N + k)*36] (6x6),
 * Bd[(b*N + k)*12] (6x2), gd[(b*N + k)*6], row-major.  The low-speed guard
 * (:143-159) acts on copies: unlike the reference, inputs are never written. */
int mpcqp_linearise_device(const mpcqp_vehicle *veh, int64_t B, int32_t N, const double *dx, int64_t x_sb,
                           int64_t x_sk, const double *du, int64_t u_sb, int64_t u_sk, double *dAd, double *dBd,
                           double *dgd, int32_t device, void *stream);

/* F1 -- the QP of mpc_increment (Control/MPC/mpc_dynamics.py:281-389) for a batch
 * sharing N, nx, nu, weights, bounds and the structural nonzeros of Ad / Bd
 * (maskA[nx*nx], maskB[nx*nu], 1 = entry may be nonzero).  Q, QN (nx x nx) and
 * R (nu x nu) are dense row-major; xmin_t / xmax_t have nx+nu entries, dumin /
 * dumax nu (+-inf allowed; clipped to +-1e30 as the osqp wrapper does).
 * Variables (x~_0..x~_N, du_0..du_{N-1}), x~ = (x, u_prev); rows [A_eq; I]. */
typedef struct mpcqp_incr_layout mpcqp_incr_layout;
int mpcqp_incr_layout_create(int32_t N, int32_t nx, int32_t nu, const double *Q, const double *QN, const double *R,
                             const double *xmin_t, const double *xmax_t, const double *dumin, const double *dumax,
                             const uint8_t *maskA, const uint8_t *maskB, int32_t device, mpcqp_incr_layout **out);
int mpcqp_incr_layout_dims(const mpcqp_incr_layout *L, int32_t *n, int32_t *m, int32_t *nnzP, int32_t *nnzA);
/* The shared pattern (P upper-triangular CSC with its constant values; A CSC) and the
 * constant parts of the per-instance arrays; any pointer may be NULL. */
int mpcqp_incr_layout_pattern(const mpcqp_incr_layout *L, int32_t *Pp, int32_t *Pi, double *Px, int32_t *Ap,
                              int32_t *Ai, double *Ax_template, double *l_template, double *u_template);
/* Per instance b: Ad/Bd/gd as produced by mpcqp_linearise_device for stages 0..N-1,
 * xt0[b*(nx+nu)] = x~(0), Xr[b*nx*(N+1)] = reference (nx rows, N+1 columns)
 * -> Ax[b*nnzA], q[b*n], l[b*m], u[b*m] for mpcqp_setup_device. */
int mpcqp_incr_assemble_device(const mpcqp_incr_layout *L, int64_t B, const double *dAd, const double *dBd,
                               const double *dgd, const double *dxt0, const double *dXr, double *dAx, double *dq,
                               double *dl, double *du, void *stream);
void mpcqp_incr_layout_free(mpcqp_incr_layout *L);

/* F1 for the LTI lateral layouts (vehicle_lateral_mpc_slack_increment.py:32-121 and its loop
 * :201-229; Control/MPC/mpc_kinematics.py:148-191 with the lateral model): their P and A
 * are the same for every instance and step (mpcqp_set_shared_matrices), and every entry of
 * the concatenated (q | l | u) is affine in the instance's parameters theta = (x0, xr) with
 * a base vector per bound regime (the script's i <= 400 / <= 900 / else schedule, :158-172):
 *     v[i] = base[regime][i] + sum_{t < T} coef[i*T + t] * theta[idx[i*T + t]]   (idx -1: none)
 * The map is built once on the host from the layout's builder (osqp_amd.mpc_device.
 * LateralAssembler); mpcqp_affine_apply_device then writes q[B*seglen0], l[B*seglen1],
 * u[B*seglen2] from theta[b*theta_stride + k] and regime[b] (NULL: regime 0; clamped to
 * [0, nregimes)), one thread per (instance, entry).  An entry with terms is the terms' sum
 * (plus its base where that is nonzero), so a product the builder forms alone is exact. */
typedef struct mpcqp_affine mpcqp_affine;
int mpcqp_affine_create(int32_t nseg, const int32_t *seglen, int32_t nregimes, int32_t T, const double *base,
                        const int32_t *idx, const double *coef, int32_t device, mpcqp_affine **out);
int mpcqp_affine_apply_device(const mpcqp_affine *a, int64_t B, const double *dtheta, int32_t theta_stride,
                              const int32_t *dregime, double *dout0, double *dout1, double *dout2, void *stream);
void mpcqp_affine_free(mpcqp_affine *a);

/* F3 -- reference_search (mpc_dynamics.py:44-90, nearest_point :30-41) for every
 * vehicle: pred[b*(N+1)*nxa + k*nxa + 0..nxa) predicted augmented states
 * -> Xr[b*6*(N+1)] (6 rows: path x, path y, yaw 0, vx 10, vy 0, r 0).  Near the
 * path's end the index holds the start of the last segment (where the reference
 * raises IndexError). */
int mpcqp_reference_search_device(int64_t B, int32_t N, int32_t nxa, int32_t npath, const double *dpath_x,
                                  const double *dpath_y, const double *dpred, double dt, double *dXr, int32_t device,
                                  void *stream);
/* F3 -- plant step and horizon shift of mpc_dynamics.main (:578-617), dynamic bicycle
 * (nx 6, nu 2): from the unscaled solutions sol[b*n] and the step's stage-0 model
 * (Ad/Bd/gd of mpcqp_linearise_device), advance x~ (xt[b*8], in/out) and write the
 * shifted predictions pred[b*(N+1)*8] and pred_du[b*(N+1)*2]. */
int mpcqp_incr_shift_device(const mpcqp_incr_layout *L, const mpcqp_vehicle *veh, int64_t B, const double *dsol,
                            const double *dAd, const double *dBd, const double *dgd, double *dxt, double *dpred,
                            double *dpdu, void *stream);
/* F3 -- warm start for the next step (cfg 5): shift a solution of
 * the incremental layout one stage forward, x[b*n], y[b*m] -> xs[b*n], ys[b*m].
 * Variable blocks x~_0..x~_N | du_0..du_{N-1} and row blocks eq_0..eq_N |
 * box_0..box_N | du-box_0..du-box_{N-1} each move k+1 -> k, the last one repeated
 * (the reference's own shift of pred_x~ / pred_du, mpc_dynamics.py:589-610, applied
 * to the primal and dual iterates).  y / ys may be NULL.  In-place is not allowed. */
int mpcqp_incr_warm_shift_device(int64_t B, int32_t N, int32_t nxa, int32_t nu, const double *dx, const double *dy,
                                 double *dxs, double *dys, int32_t device, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* MPCQP_H */
