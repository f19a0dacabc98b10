/*
 * osqp_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the OSQP 0.6.x operator-splitting QP algorithm, used as the
 * parity oracle for the MI355X solver in python-mpc_amd/ and as the CPU baseline
 * leg of bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library.  It is never linked into the product.
 *
 * What it restates (the reference calls it through `import osqp`; OSQP is a
 * third-party dependency that the reference does not vendor and that is absent
 * offline):
 *   call sites  vehicle_lateral_mpc_slack_increment.py:118,121,237,248,269
 *               Control/MPC/mpc_kinematics.py:194-198, mpc_dynamics.py:392-396, ...
 *   algorithm   published OSQP 0.6 (Stellato et al., "OSQP: an operator splitting
 *               solver for quadratic programs", Math. Prog. Comp. 2020), defaults:
 *               rho 0.1, sigma 1e-6, alpha 1.6, eps 1e-3, max_iter 4000, scaling 10,
 *               check_termination 25, adaptive rho (tolerance 5), polish off (when
 *               enabled: OSQP 0.6 polish.c -- active-set guess, reduced quasi-definite
 *               KKT with delta regularisation, iterative refinement, acceptance test).
 *
 * Parity status: OSQP outputs are not available in this environment, so iterate
 * parity against OSQP itself is UNPINNED.  The restatement is pinned by
 * (i) QP data captured from the reference's own assembly code (tests/golden/),
 * (ii) KKT optimality certificates at tight eps (tests/test_oracle.py), and
 * (iii) an independent dense numpy restatement (tests/osqp_dense_ref.py).
 *
 * One deliberate, documented choice: OSQP PyPI wheels are built with PROFILING,
 * where adaptive_rho_interval=0 means "derive from wall-clock setup time" (not
 * deterministic).  This oracle (and the GPU solver) use the non-profiling rule
 * interval = 4 * check_termination = 100, i.e. it equals OSQP run with
 * adaptive_rho_interval=100 set explicitly.
 */
#ifndef OSQP_ORACLE_H
#define OSQP_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

/* status values, identical to OSQP's constants.h */
#define ORC_DUAL_INFEASIBLE_INACCURATE 4
#define ORC_PRIMAL_INFEASIBLE_INACCURATE 3
#define ORC_SOLVED_INACCURATE 2
#define ORC_SOLVED 1
#define ORC_MAX_ITER_REACHED (-2)
#define ORC_PRIMAL_INFEASIBLE (-3)
#define ORC_DUAL_INFEASIBLE (-4)
#define ORC_SIGINT (-5)
#define ORC_TIME_LIMIT_REACHED (-6)
#define ORC_NON_CVX (-7)
#define ORC_UNSOLVED (-10)

/* setup error codes (OSQP error_flags) */
#define ORC_DATA_VALIDATION_ERROR 1
#define ORC_SETTINGS_VALIDATION_ERROR 2
#define ORC_LINSYS_SOLVER_INIT_ERROR 4
#define ORC_NONCVX_ERROR 5
#define ORC_MEM_ALLOC_ERROR 6

typedef struct {
    double rho, sigma, alpha;
    double eps_abs, eps_rel, eps_prim_inf, eps_dual_inf;
    double adaptive_rho_tolerance, adaptive_rho_fraction;
    int max_iter, scaling, check_termination, warm_start;
    int adaptive_rho, adaptive_rho_interval, scaled_termination;
    double delta;                   /* polish regularisation (OSQP default 1e-6) */
    int polish, polish_refine_iter; /* polish off / 3 refinement steps by default */
} orc_settings;

typedef struct {
    int iter, status_val, rho_updates;
    double obj_val, pri_res, dua_res, rho_estimate;
    int status_polish;              /* 0 not run, 1 polished solution taken, -1 rejected */
} orc_info;

typedef struct orc_work orc_work;

void orc_default_settings(orc_settings *s);

/* P: upper-triangular CSC (n x n), A: CSC (m x n), 0-based int32 indices.
 * l/u may hold +-inf or +-1e30.  Returns 0 or an ORC_*_ERROR code. */
int orc_setup(orc_work **out, int n, int m,
              const int *Pp, const int *Pi, const double *Px, const double *q,
              const int *Ap, const int *Ai, const double *Ax,
              const double *l, const double *u, const orc_settings *s);
int orc_update_lin_cost(orc_work *w, const double *q);
int orc_update_bounds(orc_work *w, const double *l, const double *u);
int orc_update_lower_bound(orc_work *w, const double *l);
int orc_update_upper_bound(orc_work *w, const double *u);
/* osqp_update_P_A: new values of P (upper triangle) and / or A, all (idx NULL) or at the
 * given value indices; NULL skips that matrix.  Unscale, update, rescale, refactor. */
int orc_update_P_A(orc_work *w, const double *Px, const int *Px_idx, int nP, const double *Ax,
                   const int *Ax_idx, int nA);
/* osqp_update_settings (the settings OSQP lets change after setup; rho via osqp_update_rho) */
int orc_update_settings(orc_work *w, const orc_settings *s, int set_rho);
int orc_warm_start(orc_work *w, const double *x, const double *y);
int orc_solve(orc_work *w);
/* x (n), y (m); certificates may be NULL */
void orc_get_solution(const orc_work *w, double *x, double *y,
                      double *prim_inf_cert, double *dual_inf_cert);
void orc_get_info(const orc_work *w, orc_info *info);
void orc_cleanup(orc_work *w);
int orc_kkt_nnz_L(const orc_work *w);

/* Batch helper: B independent instances sharing one sparsity pattern, each
 * run as a fresh setup()+solve() (the Control/MPC call pattern).  Per-instance
 * value arrays are laid out instance-major.  Uses `nthreads` POSIX threads
 * (static contiguous slices).  Returns 0 or the first setup error code. */
int orc_solve_batch(int B, int n, int m,
                    const int *Pp, const int *Pi, const double *Px_b, const double *q_b,
                    const int *Ap, const int *Ai, const double *Ax_b,
                    const double *l_b, const double *u_b, const orc_settings *s,
                    double *x_out, double *y_out, int *status, int *iters,
                    int nthreads);
/* Same, each instance warm-started from x0_b[b*n], y0_b[b*m] (osqp_warm_start) after
 * its setup; NULL x0_b / y0_b = cold. */
int orc_solve_batch_warm(int B, int n, int m,
                         const int *Pp, const int *Pi, const double *Px_b, const double *q_b,
                         const int *Ap, const int *Ai, const double *Ax_b,
                         const double *l_b, const double *u_b, const double *x0_b, const double *y0_b,
                         const orc_settings *s, double *x_out, double *y_out, int *status, int *iters,
                         int nthreads);

/* Same, and phase_s[0] / phase_s[1] (may be NULL) receive the thread-seconds spent in
 * setup (+ warm start) and in solve, summed over the threads (bench.py's CPU baseline). */
int orc_solve_batch_timed(int B, int n, int m,
                          const int *Pp, const int *Pi, const double *Px_b, const double *q_b,
                          const int *Ap, const int *Ai, const double *Ax_b,
                          const double *l_b, const double *u_b, const double *x0_b, const double *y0_b,
                          const orc_settings *s, double *x_out, double *y_out, int *status, int *iters,
                          int nthreads, double *phase_s);

#ifdef __cplusplus
}
#endif
#endif
