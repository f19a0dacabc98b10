/*
 * osqp_oracle.c -- TEST INFRASTRUCTURE ONLY (see osqp_oracle.h).
 *
 * CPU restatement of OSQP 0.6.x: Ruiz equilibration, rho-vector classes,
 * quasi-definite KKT  [[P + sigma I, A'], [A, -diag(1/rho)]]  factored as
 * L D L' (minimum-degree ordering + up-looking elimination-tree LDL, the
 * algorithm QDLDL implements), the alpha-relaxed ADMM loop, termination and
 * infeasibility tests every check_termination iterations, adaptive rho with
 * refactorisation, unscaling.  Function names follow OSQP's so the restatement
 * can be read side by side with the published algorithm; no OSQP source is in
 * this environment.
 *
 * Reference call sites restated here:
 *   setup   vehicle_lateral_mpc_slack_increment.py:118-121,
 *           Control/MPC/mpc_dynamics.py:392-393, mpc_kinematics.py:194-195
 *   update  vehicle_lateral_mpc_slack_increment.py:237,269
 *   solve   vehicle_lateral_mpc_slack_increment.py:248, mpc_dynamics.py:396
 */
#include "osqp_oracle.h"

#include <math.h>
#include <pthread.h>
#include <time.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OSQP_INFTY 1e30
#define MIN_SCALING 1e-4
#define MAX_SCALING 1e4
#define RHO_MIN 1e-6
#define RHO_MAX 1e6
#define RHO_TOL 1e-4
#define RHO_EQ_OVER_RHO_INEQ 1e3
#define DIVISION_TOL (1.0 / OSQP_INFTY)
#define ADAPTIVE_RHO_MULTIPLE_TERMINATION 4
#define ADAPTIVE_RHO_FIXED 100

static double dmax(double a, double b) { return a > b ? a : b; }
static double dmin(double a, double b) { return a < b ? a : b; }

/* ------------------------------------------------------------------ KKT -- */
typedef struct {
    int N, n, m;
    int *perm;        /* perm[k] = original index of pivot k */
    int *pinv;        /* pinv[orig] = k */
    int *Kp, *Ki;     /* permuted upper-triangular KKT, CSC */
    double *Kx;
    int *rho_pos;     /* Kx index of the -1/rho_i diagonal, i < m */
    int *etree, *Lnz, *Lp, *Li;
    double *Lx, *Dv, *Dinv;
    int *iw;          /* 3N ints workspace */
    double *fw;       /* N doubles workspace */
    double *bp;       /* N doubles */
} kkt_t;

static void kkt_free(kkt_t *k) {
    if (!k) return;
    free(k->perm); free(k->pinv); free(k->Kp); free(k->Ki); free(k->Kx);
    free(k->rho_pos); free(k->etree); free(k->Lnz); free(k->Lp); free(k->Li);
    free(k->Lx); free(k->Dv); free(k->Dinv); free(k->iw); free(k->fw); free(k->bp);
    free(k);
}

/* Minimum-degree ordering on the explicit elimination graph (bitsets).  Any
 * fill-reducing order gives the same factorisation in exact arithmetic; OSQP
 * uses AMD, this is the plain (non-approximate) minimum-degree rule. */
static int min_degree(int N, const int *cp, const int *ri, int *perm) {
    int W = (N + 63) / 64;
    uint64_t *adj = (uint64_t *)calloc((size_t)N * W, sizeof(uint64_t));
    int *deg = (int *)calloc(N, sizeof(int));
    char *done = (char *)calloc(N, 1);
    int *nb = (int *)malloc(sizeof(int) * (N > 0 ? N : 1));
    if (!adj || !deg || !done || !nb) { free(adj); free(deg); free(done); free(nb); return -1; }
    for (int j = 0; j < N; ++j)
        for (int p = cp[j]; p < cp[j + 1]; ++p) {
            int i = ri[p];
            if (i == j) continue;
            adj[(size_t)i * W + j / 64] |= 1ull << (j % 64);
            adj[(size_t)j * W + i / 64] |= 1ull << (i % 64);
        }
    for (int i = 0; i < N; ++i) {
        int d = 0;
        for (int w = 0; w < W; ++w) d += __builtin_popcountll(adj[(size_t)i * W + w]);
        deg[i] = d;
    }
    for (int k = 0; k < N; ++k) {
        int v = -1;
        for (int i = 0; i < N; ++i)
            if (!done[i] && (v < 0 || deg[i] < deg[v])) v = i;
        perm[k] = v;
        done[v] = 1;
        uint64_t *av = adj + (size_t)v * W;
        int cnt = 0;
        for (int w = 0; w < W; ++w) {
            uint64_t bits = av[w];
            while (bits) {
                int b = __builtin_ctzll(bits);
                bits &= bits - 1;
                nb[cnt++] = w * 64 + b;
            }
        }
        for (int t = 0; t < cnt; ++t) {
            int u = nb[t];
            uint64_t *au = adj + (size_t)u * W;
            for (int w = 0; w < W; ++w) au[w] |= av[w];
            au[u / 64] &= ~(1ull << (u % 64));
            au[v / 64] &= ~(1ull << (v % 64));
            int d = 0;
            for (int w = 0; w < W; ++w) d += __builtin_popcountll(au[w]);
            deg[u] = d;
        }
    }
    free(adj); free(deg); free(done); free(nb);
    return 0;
}

/* elimination tree + column counts of L for an upper-triangular CSC matrix
 * (the QDLDL_etree recurrence). returns sum of counts or -1 */
static int ldl_etree(int N, const int *Ap, const int *Ai, int *work, int *Lnz, int *etree) {
    for (int i = 0; i < N; ++i) { work[i] = 0; Lnz[i] = 0; etree[i] = -1; }
    for (int j = 0; j < N; ++j) {
        work[j] = j;
        for (int p = Ap[j]; p < Ap[j + 1]; ++p) {
            int i = Ai[p];
            if (i > j) return -1;
            while (work[i] != j) {
                if (etree[i] == -1) etree[i] = j;
                Lnz[i]++;
                work[i] = j;
                i = etree[i];
            }
        }
    }
    int s = 0;
    for (int i = 0; i < N; ++i) s += Lnz[i];
    return s;
}

/* up-looking numeric LDL'. returns number of positive pivots, or -1 on a zero
 * pivot. */
static int ldl_numeric(kkt_t *k) {
    int N = k->N;
    int *flag = k->iw, *pattern = k->iw + N, *nfill = k->iw + 2 * N;
    double *y = k->fw;
    int npos = 0;
    k->Lp[0] = 0;
    for (int i = 0; i < N; ++i) {
        k->Lp[i + 1] = k->Lp[i] + k->Lnz[i];
        flag[i] = -1; nfill[i] = 0; y[i] = 0.0;
    }
    for (int j = 0; j < N; ++j) {
        int top = N;
        flag[j] = j;
        for (int p = k->Kp[j]; p < k->Kp[j + 1]; ++p) {
            int i = k->Ki[p];
            y[i] += k->Kx[p];
            int len = 0;
            while (flag[i] != j) {
                pattern[len++] = i;
                flag[i] = j;
                i = k->etree[i];
            }
            while (len > 0) pattern[--top] = pattern[--len];
        }
        double d = y[j];
        y[j] = 0.0;
        for (int t = top; t < N; ++t) {
            int i = pattern[t];
            double yi = y[i];
            y[i] = 0.0;
            int p0 = k->Lp[i], p1 = k->Lp[i] + nfill[i];
            for (int p = p0; p < p1; ++p) y[k->Li[p]] -= k->Lx[p] * yi;
            double lji = yi / k->Dv[i];
            d -= lji * yi;
            k->Li[p1] = j;
            k->Lx[p1] = lji;
            nfill[i]++;
        }
        if (d == 0.0) return -1;
        k->Dv[j] = d;
        k->Dinv[j] = 1.0 / d;
        if (d > 0.0) npos++;
    }
    return npos;
}

/* build permuted KKT, order, symbolic + numeric factor.  P upper CSC (n), A CSC (m x n). */
static int kkt_init(kkt_t **out, int n, int m, const int *Pp, const int *Pi, const double *Px,
                    const int *Ap, const int *Ai, const double *Ax, double sigma,
                    const double *rho_inv) {
    kkt_t *k = (kkt_t *)calloc(1, sizeof(kkt_t));
    if (!k) return ORC_MEM_ALLOC_ERROR;
    int N = n + m;
    k->N = N; k->n = n; k->m = m;
    int nnzP = Pp[n], nnzA = Ap[n];
    /* original-index upper-triangular KKT as triplets (col-major CSC build) */
    int cap = nnzP + n + nnzA + m;
    int *tr = (int *)malloc(sizeof(int) * cap), *tc = (int *)malloc(sizeof(int) * cap);
    double *tv = (double *)malloc(sizeof(double) * cap);
    int *tag = (int *)malloc(sizeof(int) * cap); /* -1: P/sigma, -2: A, i>=0: rho diag of row i */
    int nt = 0;
    for (int j = 0; j < n; ++j) {
        int hasdiag = 0;
        for (int p = Pp[j]; p < Pp[j + 1]; ++p) {
            int i = Pi[p];
            double v = Px[p];
            if (i == j) { v += sigma; hasdiag = 1; }
            tr[nt] = i; tc[nt] = j; tv[nt] = v; tag[nt] = -1; nt++;
        }
        if (!hasdiag) { tr[nt] = j; tc[nt] = j; tv[nt] = sigma; tag[nt] = -1; nt++; }
    }
    for (int j = 0; j < n; ++j)
        for (int p = Ap[j]; p < Ap[j + 1]; ++p) { /* A(i,j) -> KKT(j, n+i), upper */
            tr[nt] = j; tc[nt] = n + Ai[p]; tv[nt] = Ax[p]; tag[nt] = -2; nt++;
        }
    for (int i = 0; i < m; ++i) { tr[nt] = n + i; tc[nt] = n + i; tv[nt] = -rho_inv[i]; tag[nt] = i; nt++; }

    /* pattern CSC in original index space for the ordering */
    int *cp = (int *)calloc(N + 1, sizeof(int)), *ri = (int *)malloc(sizeof(int) * (nt ? nt : 1));
    for (int t = 0; t < nt; ++t) cp[tc[t] + 1]++;
    for (int j = 0; j < N; ++j) cp[j + 1] += cp[j];
    {
        int *pos = (int *)malloc(sizeof(int) * (N + 1));
        memcpy(pos, cp, sizeof(int) * (N + 1));
        for (int t = 0; t < nt; ++t) ri[pos[tc[t]]++] = tr[t];
        free(pos);
    }
    k->perm = (int *)malloc(sizeof(int) * N);
    k->pinv = (int *)malloc(sizeof(int) * N);
    if (min_degree(N, cp, ri, k->perm)) { free(cp); free(ri); kkt_free(k); return ORC_MEM_ALLOC_ERROR; }
    for (int i = 0; i < N; ++i) k->pinv[k->perm[i]] = i;
    free(cp); free(ri);

    /* permuted upper triangular */
    k->Kp = (int *)calloc(N + 1, sizeof(int));
    k->Ki = (int *)malloc(sizeof(int) * nt);
    k->Kx = (double *)malloc(sizeof(double) * nt);
    k->rho_pos = (int *)malloc(sizeof(int) * (m ? m : 1));
    for (int t = 0; t < nt; ++t) {
        int a = k->pinv[tr[t]], b = k->pinv[tc[t]];
        int c = a > b ? a : b;
        k->Kp[c + 1]++;
    }
    for (int j = 0; j < N; ++j) k->Kp[j + 1] += k->Kp[j];
    {
        int *pos = (int *)malloc(sizeof(int) * (N + 1));
        memcpy(pos, k->Kp, sizeof(int) * (N + 1));
        for (int t = 0; t < nt; ++t) {
            int a = k->pinv[tr[t]], b = k->pinv[tc[t]];
            int r = a < b ? a : b, c = a > b ? a : b;
            int q = pos[c]++;
            k->Ki[q] = r; k->Kx[q] = tv[t];
            if (tag[t] >= 0) k->rho_pos[tag[t]] = q;
        }
        free(pos);
    }
    free(tr); free(tc); free(tv); free(tag);

    k->etree = (int *)malloc(sizeof(int) * N);
    k->Lnz = (int *)malloc(sizeof(int) * N);
    k->iw = (int *)malloc(sizeof(int) * 3 * N);
    k->fw = (double *)malloc(sizeof(double) * N);
    k->bp = (double *)malloc(sizeof(double) * N);
    k->Lp = (int *)malloc(sizeof(int) * (N + 1));
    k->Dv = (double *)malloc(sizeof(double) * N);
    k->Dinv = (double *)malloc(sizeof(double) * N);
    int sumL = ldl_etree(N, k->Kp, k->Ki, k->iw, k->Lnz, k->etree);
    if (sumL < 0) { kkt_free(k); return ORC_LINSYS_SOLVER_INIT_ERROR; }
    k->Li = (int *)malloc(sizeof(int) * (sumL ? sumL : 1));
    k->Lx = (double *)malloc(sizeof(double) * (sumL ? sumL : 1));
    int npos = ldl_numeric(k);
    if (npos < 0) { kkt_free(k); return ORC_LINSYS_SOLVER_INIT_ERROR; }
    if (npos < n) { kkt_free(k); return ORC_NONCVX_ERROR; }
    *out = k;
    return 0;
}

static int kkt_update_rho(kkt_t *k, const double *rho_inv) {
    for (int i = 0; i < k->m; ++i) k->Kx[k->rho_pos[i]] = -rho_inv[i];
    int npos = ldl_numeric(k);
    return (npos < k->n) ? -1 : 0;
}

/* solve KKT * sol = b (b original order, overwritten by sol) */
static void kkt_solve(kkt_t *k, double *b) {
    int N = k->N;
    double *x = k->bp;
    for (int i = 0; i < N; ++i) x[i] = b[k->perm[i]];
    for (int j = 0; j < N; ++j) {
        double xj = x[j];
        for (int p = k->Lp[j]; p < k->Lp[j + 1]; ++p) x[k->Li[p]] -= k->Lx[p] * xj;
    }
    for (int j = 0; j < N; ++j) x[j] *= k->Dinv[j];
    for (int j = N - 1; j >= 0; --j) {
        double s = x[j];
        for (int p = k->Lp[j]; p < k->Lp[j + 1]; ++p) s -= k->Lx[p] * x[k->Li[p]];
        x[j] = s;
    }
    for (int i = 0; i < N; ++i) b[k->perm[i]] = x[i];
}

/* ------------------------------------------------------------ workspace -- */
struct orc_work {
    int n, m;
    int *Pp, *Pi, *Ap, *Ai;
    double *Px, *Ax, *q, *l, *u;
    double *D, *Dinv, *E, *Einv, c, cinv;
    double *rho_vec, *rho_inv_vec;
    int *constr_type;
    double *x, *y, *z, *xz_tilde, *x_prev, *z_prev;
    double *Axv, *Pxv, *Aty, *delta_y, *Atdelta_y, *delta_x, *Pdelta_x, *Adelta_x;
    double *sol_x, *sol_y;
    kkt_t *kkt;
    orc_settings set;
    orc_info info;
};

void orc_default_settings(orc_settings *s) {
    s->delta = 1e-6; s->polish = 0; s->polish_refine_iter = 3;
    s->rho = 0.1; s->sigma = 1e-6; s->alpha = 1.6;
    s->eps_abs = 1e-3; s->eps_rel = 1e-3; s->eps_prim_inf = 1e-4; s->eps_dual_inf = 1e-4;
    s->adaptive_rho_tolerance = 5.0; s->adaptive_rho_fraction = 0.4;
    s->max_iter = 4000; s->scaling = 10; s->check_termination = 25; s->warm_start = 1;
    s->adaptive_rho = 1; s->adaptive_rho_interval = 0; s->scaled_termination = 0;
}

/* ---- small linear algebra on CSC (OSQP lin_alg.c semantics) ---- */
static double vec_norm_inf(const double *v, int l) {
    double r = 0.0;
    for (int i = 0; i < l; ++i) r = dmax(r, fabs(v[i]));
    return r;
}
static double vec_scaled_norm_inf(const double *S, const double *v, int l) {
    double r = 0.0;
    for (int i = 0; i < l; ++i) r = dmax(r, fabs(S[i] * v[i]));
    return r;
}
/* y = A x (plus_eq: y += A x) */
static void mat_vec(int ncol, const int *Ap, const int *Ai, const double *Ax, int nrow,
                    const double *x, double *y, int plus_eq) {
    if (!plus_eq) for (int i = 0; i < nrow; ++i) y[i] = 0.0;
    for (int j = 0; j < ncol; ++j)
        for (int p = Ap[j]; p < Ap[j + 1]; ++p) y[Ai[p]] += Ax[p] * x[j];
}
/* y = A' x ; skip_diag for symmetric-triu use */
static void mat_tpose_vec(int ncol, const int *Ap, const int *Ai, const double *Ax,
                          const double *x, double *y, int plus_eq, int skip_diag) {
    if (!plus_eq) for (int j = 0; j < ncol; ++j) y[j] = 0.0;
    for (int j = 0; j < ncol; ++j)
        for (int p = Ap[j]; p < Ap[j + 1]; ++p) {
            if (skip_diag && Ai[p] == j) continue;
            y[j] += Ax[p] * x[Ai[p]];
        }
}
/* full symmetric P x from upper triangle */
static void sym_mat_vec(const orc_work *w, const double *x, double *y) {
    mat_vec(w->n, w->Pp, w->Pi, w->Px, w->n, x, y, 0);
    mat_tpose_vec(w->n, w->Pp, w->Pi, w->Px, x, y, 1, 1);
}
static double quad_form(const orc_work *w, const double *x) {
    double r = 0.0;
    for (int j = 0; j < w->n; ++j)
        for (int p = w->Pp[j]; p < w->Pp[j + 1]; ++p) {
            int i = w->Pi[p];
            if (i == j) r += 0.5 * w->Px[p] * x[i] * x[i];
            else if (i < j) r += w->Px[p] * x[i] * x[j];
        }
    return r;
}
static void limit_scaling(double *D, int n) {
    for (int i = 0; i < n; ++i) {
        D[i] = D[i] < MIN_SCALING ? 1.0 : D[i];
        D[i] = D[i] > MAX_SCALING ? MAX_SCALING : D[i];
    }
}

/* ---- scaling.c: scale_data ---- */
static void scale_data(orc_work *w) {
    int n = w->n, m = w->m;
    double *Dt = (double *)malloc(sizeof(double) * (n ? n : 1));
    double *DtA = (double *)malloc(sizeof(double) * (n ? n : 1));
    double *Et = (double *)malloc(sizeof(double) * (m ? m : 1));
    w->c = 1.0;
    for (int i = 0; i < n; ++i) { w->D[i] = 1.0; w->Dinv[i] = 1.0; }
    for (int i = 0; i < m; ++i) { w->E[i] = 1.0; w->Einv[i] = 1.0; }
    for (int it = 0; it < w->set.scaling; ++it) {
        /* compute_inf_norm_cols_KKT */
        for (int j = 0; j < n; ++j) { Dt[j] = 0.0; DtA[j] = 0.0; }
        for (int j = 0; j < n; ++j)
            for (int p = w->Pp[j]; p < w->Pp[j + 1]; ++p) {
                int i = w->Pi[p];
                double a = fabs(w->Px[p]);
                Dt[j] = dmax(a, Dt[j]);
                if (i != j) Dt[i] = dmax(a, Dt[i]);
            }
        for (int j = 0; j < n; ++j)
            for (int p = w->Ap[j]; p < w->Ap[j + 1]; ++p) DtA[j] = dmax(fabs(w->Ax[p]), DtA[j]);
        for (int j = 0; j < n; ++j) Dt[j] = dmax(Dt[j], DtA[j]);
        for (int i = 0; i < m; ++i) Et[i] = 0.0;
        for (int j = 0; j < n; ++j)
            for (int p = w->Ap[j]; p < w->Ap[j + 1]; ++p) {
                int i = w->Ai[p];
                Et[i] = dmax(fabs(w->Ax[p]), Et[i]);
            }
        limit_scaling(Dt, n);
        limit_scaling(Et, m);
        for (int j = 0; j < n; ++j) Dt[j] = 1.0 / sqrt(Dt[j]);
        for (int i = 0; i < m; ++i) Et[i] = 1.0 / sqrt(Et[i]);
        /* P <- Dt P Dt ; A <- Et A Dt ; q <- Dt q  (mat_premult_diag, then mat_postmult_diag:
         * two roundings per entry, in that order) */
        for (int j = 0; j < n; ++j)
            for (int p = w->Pp[j]; p < w->Pp[j + 1]; ++p) { w->Px[p] *= Dt[w->Pi[p]]; w->Px[p] *= Dt[j]; }
        for (int j = 0; j < n; ++j)
            for (int p = w->Ap[j]; p < w->Ap[j + 1]; ++p) { w->Ax[p] *= Et[w->Ai[p]]; w->Ax[p] *= Dt[j]; }
        for (int j = 0; j < n; ++j) w->q[j] *= Dt[j];
        for (int j = 0; j < n; ++j) w->D[j] *= Dt[j];
        for (int i = 0; i < m; ++i) w->E[i] *= Et[i];
        /* cost normalisation */
        for (int j = 0; j < n; ++j) Dt[j] = 0.0;
        for (int j = 0; j < n; ++j)
            for (int p = w->Pp[j]; p < w->Pp[j + 1]; ++p) {
                int i = w->Pi[p];
                double a = fabs(w->Px[p]);
                Dt[j] = dmax(a, Dt[j]);
                if (i != j) Dt[i] = dmax(a, Dt[i]);
            }
        double ct = 0.0;
        for (int j = 0; j < n; ++j) ct += Dt[j];
        ct /= (double)n;
        double nq = vec_norm_inf(w->q, n);
        limit_scaling(&nq, 1);
        ct = dmax(ct, nq);
        limit_scaling(&ct, 1);
        ct = 1.0 / ct;
        for (int p = 0; p < w->Pp[n]; ++p) w->Px[p] *= ct;
        for (int j = 0; j < n; ++j) w->q[j] *= ct;
        w->c *= ct;
    }
    w->cinv = 1.0 / w->c;
    for (int j = 0; j < n; ++j) w->Dinv[j] = 1.0 / w->D[j];
    for (int i = 0; i < m; ++i) w->Einv[i] = 1.0 / w->E[i];
    for (int i = 0; i < m; ++i) { w->l[i] *= w->E[i]; w->u[i] *= w->E[i]; }
    free(Dt); free(DtA); free(Et);
}

static void set_rho_vec(orc_work *w) {
    w->set.rho = dmin(dmax(w->set.rho, RHO_MIN), RHO_MAX);
    for (int i = 0; i < w->m; ++i) {
        if (w->l[i] < -OSQP_INFTY * MIN_SCALING && w->u[i] > OSQP_INFTY * MIN_SCALING) {
            w->constr_type[i] = -1;
            w->rho_vec[i] = RHO_MIN;
        } else if (w->u[i] - w->l[i] < RHO_TOL) {
            w->constr_type[i] = 1;
            w->rho_vec[i] = RHO_EQ_OVER_RHO_INEQ * w->set.rho;
        } else {
            w->constr_type[i] = 0;
            w->rho_vec[i] = w->set.rho;
        }
        w->rho_inv_vec[i] = 1.0 / w->rho_vec[i];
    }
}

static int update_rho_vec(orc_work *w) {
    int changed = 0;
    for (int i = 0; i < w->m; ++i) {
        if (w->l[i] < -OSQP_INFTY * MIN_SCALING && w->u[i] > OSQP_INFTY * MIN_SCALING) {
            if (w->constr_type[i] != -1) {
                w->constr_type[i] = -1; w->rho_vec[i] = RHO_MIN; w->rho_inv_vec[i] = 1.0 / RHO_MIN; changed = 1;
            }
        } else if (w->u[i] - w->l[i] < RHO_TOL) {
            if (w->constr_type[i] != 1) {
                w->constr_type[i] = 1; w->rho_vec[i] = RHO_EQ_OVER_RHO_INEQ * w->set.rho;
                w->rho_inv_vec[i] = 1.0 / w->rho_vec[i]; changed = 1;
            }
        } else {
            if (w->constr_type[i] != 0) {
                w->constr_type[i] = 0; w->rho_vec[i] = w->set.rho; w->rho_inv_vec[i] = 1.0 / w->set.rho; changed = 1;
            }
        }
    }
    if (changed) return kkt_update_rho(w->kkt, w->rho_inv_vec);
    return 0;
}

static void reset_info(orc_work *w) { w->info.status_val = ORC_UNSOLVED; }

static double *dalloc(int k) { return (double *)calloc(k > 0 ? k : 1, sizeof(double)); }

void orc_cleanup(orc_work *w) {
    if (!w) return;
    free(w->Pp); free(w->Pi); free(w->Ap); free(w->Ai); free(w->Px); free(w->Ax);
    free(w->q); free(w->l); free(w->u); free(w->D); free(w->Dinv); free(w->E); free(w->Einv);
    free(w->rho_vec); free(w->rho_inv_vec); free(w->constr_type);
    free(w->x); free(w->y); free(w->z); free(w->xz_tilde); free(w->x_prev); free(w->z_prev);
    free(w->Axv); free(w->Pxv); free(w->Aty); free(w->delta_y); free(w->Atdelta_y);
    free(w->delta_x); free(w->Pdelta_x); free(w->Adelta_x); free(w->sol_x); free(w->sol_y);
    kkt_free(w->kkt);
    free(w);
}

int orc_setup(orc_work **out, int n, int m, const int *Pp, const int *Pi, const double *Px,
              const double *q, const int *Ap, const int *Ai, const double *Ax,
              const double *l, const double *u, const orc_settings *s) {
    *out = NULL;
    /* validate_data */
    if (n <= 0 || m < 0) return ORC_DATA_VALIDATION_ERROR;
    for (int j = 0; j < n; ++j)
        for (int p = Pp[j]; p < Pp[j + 1]; ++p)
            if (Pi[p] > j || Pi[p] < 0) return ORC_DATA_VALIDATION_ERROR; /* P not upper triangular */
    for (int i = 0; i < m; ++i)
        if (l[i] > u[i]) return ORC_DATA_VALIDATION_ERROR;
    /* validate_settings (subset) */
    if (s->rho <= 0 || s->sigma <= 0 || s->max_iter <= 0 || s->eps_abs < 0 || s->eps_rel < 0 ||
        (s->eps_abs == 0 && s->eps_rel == 0) || s->eps_prim_inf <= 0 || s->eps_dual_inf <= 0 ||
        s->alpha <= 0 || s->alpha >= 2 || s->scaling < 0 || s->check_termination < 0 ||
        s->adaptive_rho_interval < 0 || s->adaptive_rho_tolerance < 1)
        return ORC_SETTINGS_VALIDATION_ERROR;
    orc_work *w = (orc_work *)calloc(1, sizeof(orc_work));
    if (!w) return ORC_MEM_ALLOC_ERROR;
    w->n = n; w->m = m; w->set = *s;
    int nnzP = Pp[n], nnzA = Ap[n];
    w->Pp = (int *)malloc(sizeof(int) * (n + 1)); memcpy(w->Pp, Pp, sizeof(int) * (n + 1));
    w->Pi = (int *)malloc(sizeof(int) * (nnzP ? nnzP : 1)); memcpy(w->Pi, Pi, sizeof(int) * nnzP);
    w->Px = dalloc(nnzP); memcpy(w->Px, Px, sizeof(double) * nnzP);
    w->Ap = (int *)malloc(sizeof(int) * (n + 1)); memcpy(w->Ap, Ap, sizeof(int) * (n + 1));
    w->Ai = (int *)malloc(sizeof(int) * (nnzA ? nnzA : 1)); memcpy(w->Ai, Ai, sizeof(int) * nnzA);
    w->Ax = dalloc(nnzA); memcpy(w->Ax, Ax, sizeof(double) * nnzA);
    w->q = dalloc(n); memcpy(w->q, q, sizeof(double) * n);
    w->l = dalloc(m); w->u = dalloc(m);
    for (int i = 0; i < m; ++i) {  /* python wrapper clips to +-OSQP_INFTY */
        w->l[i] = dmax(l[i], -OSQP_INFTY);
        w->u[i] = dmin(u[i], OSQP_INFTY);
    }
    w->D = dalloc(n); w->Dinv = dalloc(n); w->E = dalloc(m); w->Einv = dalloc(m);
    w->rho_vec = dalloc(m); w->rho_inv_vec = dalloc(m);
    w->constr_type = (int *)calloc(m ? m : 1, sizeof(int));
    w->x = dalloc(n); w->y = dalloc(m); w->z = dalloc(m); w->xz_tilde = dalloc(n + m);
    w->x_prev = dalloc(n); w->z_prev = dalloc(m);
    w->Axv = dalloc(m); w->Pxv = dalloc(n); w->Aty = dalloc(n);
    w->delta_y = dalloc(m); w->Atdelta_y = dalloc(n); w->delta_x = dalloc(n);
    w->Pdelta_x = dalloc(n); w->Adelta_x = dalloc(m);
    w->sol_x = dalloc(n); w->sol_y = dalloc(m);
    if (w->set.scaling) {
        scale_data(w);
    } else {
        w->c = 1.0; w->cinv = 1.0;
        for (int i = 0; i < n; ++i) { w->D[i] = 1.0; w->Dinv[i] = 1.0; }
        for (int i = 0; i < m; ++i) { w->E[i] = 1.0; w->Einv[i] = 1.0; }
    }
    set_rho_vec(w);
    int e = kkt_init(&w->kkt, n, m, w->Pp, w->Pi, w->Px, w->Ap, w->Ai, w->Ax, w->set.sigma,
                     w->rho_inv_vec);
    if (e) { orc_cleanup(w); return e; }
    /* non-profiling rule for adaptive_rho_interval == 0 (pinned, see header), resolved here as
     * osqp_setup does in builds without profiling: a later update_settings(check_termination=)
     * does not move it */
    if (w->set.adaptive_rho && !w->set.adaptive_rho_interval) {
        if (w->set.check_termination)
            w->set.adaptive_rho_interval = ADAPTIVE_RHO_MULTIPLE_TERMINATION * w->set.check_termination;
        else
            w->set.adaptive_rho_interval = ADAPTIVE_RHO_FIXED;
    }
    w->info.status_val = ORC_UNSOLVED;
    w->info.rho_updates = 0;
    w->info.rho_estimate = w->set.rho;
    *out = w;
    return 0;
}

/* ---- osqp_api_functions: updates ---- */
int orc_update_lin_cost(orc_work *w, const double *q) {
    memcpy(w->q, q, sizeof(double) * w->n);
    if (w->set.scaling) {
        for (int j = 0; j < w->n; ++j) w->q[j] *= w->D[j];
        for (int j = 0; j < w->n; ++j) w->q[j] *= w->c;
    }
    reset_info(w);
    return 0;
}
int orc_update_bounds(orc_work *w, const double *l, const double *u) {
    for (int i = 0; i < w->m; ++i)
        if (dmax(l[i], -OSQP_INFTY) > dmin(u[i], OSQP_INFTY)) return ORC_DATA_VALIDATION_ERROR;
    for (int i = 0; i < w->m; ++i) {
        w->l[i] = dmax(l[i], -OSQP_INFTY);
        w->u[i] = dmin(u[i], OSQP_INFTY);
        if (w->set.scaling) { w->l[i] *= w->E[i]; w->u[i] *= w->E[i]; }
    }
    reset_info(w);
    return update_rho_vec(w);
}
int orc_update_lower_bound(orc_work *w, const double *l) {
    for (int i = 0; i < w->m; ++i) {
        double li = dmax(l[i], -OSQP_INFTY);
        if (w->set.scaling) li *= w->E[i];
        if (li > w->u[i]) return ORC_DATA_VALIDATION_ERROR;
    }
    for (int i = 0; i < w->m; ++i) {
        w->l[i] = dmax(l[i], -OSQP_INFTY);
        if (w->set.scaling) w->l[i] *= w->E[i];
    }
    reset_info(w);
    return update_rho_vec(w);
}
int orc_update_upper_bound(orc_work *w, const double *u) {
    for (int i = 0; i < w->m; ++i) {
        double ui = dmin(u[i], OSQP_INFTY);
        if (w->set.scaling) ui *= w->E[i];
        if (w->l[i] > ui) return ORC_DATA_VALIDATION_ERROR;
    }
    for (int i = 0; i < w->m; ++i) {
        w->u[i] = dmin(u[i], OSQP_INFTY);
        if (w->set.scaling) w->u[i] *= w->E[i];
    }
    reset_info(w);
    return update_rho_vec(w);
}
int orc_warm_start(orc_work *w, const double *x, const double *y) {
    w->set.warm_start = 1;
    memcpy(w->x, x, sizeof(double) * w->n);
    memcpy(w->y, y, sizeof(double) * w->m);
    if (w->set.scaling) {
        for (int j = 0; j < w->n; ++j) w->x[j] *= w->Dinv[j];
        for (int i = 0; i < w->m; ++i) { w->y[i] *= w->Einv[i]; w->y[i] *= w->c; }  /* vec_ew_prod, vec_mult_scalar */
    }
    mat_vec(w->n, w->Ap, w->Ai, w->Ax, w->m, w->x, w->z, 0);
    return 0;
}

/* ---- scaling.c: unscale_data (OSQP 0.6), used by the matrix updates ----
 * P <- cinv Dinv P Dinv (mat_mult_scalar, mat_premult_diag, mat_postmult_diag),
 * q <- Dinv (cinv q), A <- Einv A Dinv, l <- Einv l, u <- Einv u: one rounding per
 * factor, in OSQP's order. */
static void unscale_data(orc_work *w) {
    int n = w->n, m = w->m;
    for (int p = 0; p < w->Pp[n]; ++p) w->Px[p] *= w->cinv;
    for (int j = 0; j < n; ++j)
        for (int p = w->Pp[j]; p < w->Pp[j + 1]; ++p) { w->Px[p] *= w->Dinv[w->Pi[p]]; w->Px[p] *= w->Dinv[j]; }
    for (int j = 0; j < n; ++j) { w->q[j] *= w->cinv; w->q[j] *= w->Dinv[j]; }
    for (int j = 0; j < n; ++j)
        for (int p = w->Ap[j]; p < w->Ap[j + 1]; ++p) { w->Ax[p] *= w->Einv[w->Ai[p]]; w->Ax[p] *= w->Dinv[j]; }
    for (int i = 0; i < m; ++i) { w->l[i] *= w->Einv[i]; w->u[i] *= w->Einv[i]; }
}

/* osqp_update_P / osqp_update_A / osqp_update_P_A (OSQP 0.6 osqp.c): unscale the data,
 * write the new values (all of them, or those at the given indices of P's upper-triangular
 * / A's CSC value arrays, in order), scale from scratch, refactor the KKT matrix with the
 * rho vector as it is, reset the status.  x, z, y and the rho vector are left as they are
 * (OSQP 0.6 keeps the iterates in the previous scaling).  Px / Ax NULL: that matrix is not
 * updated; *_idx NULL: all nnz values. */
int orc_update_P_A(orc_work *w, const double *Px, const int *Px_idx, int nP, const double *Ax,
                   const int *Ax_idx, int nA) {
    int nnzP = w->Pp[w->n], nnzA = w->Ap[w->n];
    if ((Px && Px_idx && (nP < 0 || nP > nnzP)) || (Ax && Ax_idx && (nA < 0 || nA > nnzA)))
        return ORC_DATA_VALIDATION_ERROR;
    if (Px_idx) for (int k = 0; k < nP; ++k) if (Px_idx[k] < 0 || Px_idx[k] >= nnzP) return ORC_DATA_VALIDATION_ERROR;
    if (Ax_idx) for (int k = 0; k < nA; ++k) if (Ax_idx[k] < 0 || Ax_idx[k] >= nnzA) return ORC_DATA_VALIDATION_ERROR;
    if (w->set.scaling) unscale_data(w);
    if (Px) {
        if (Px_idx) for (int k = 0; k < nP; ++k) w->Px[Px_idx[k]] = Px[k];
        else memcpy(w->Px, Px, sizeof(double) * nnzP);
    }
    if (Ax) {
        if (Ax_idx) for (int k = 0; k < nA; ++k) w->Ax[Ax_idx[k]] = Ax[k];
        else memcpy(w->Ax, Ax, sizeof(double) * nnzA);
    }
    if (w->set.scaling) scale_data(w);
    kkt_free(w->kkt);
    w->kkt = NULL;
    int e = kkt_init(&w->kkt, w->n, w->m, w->Pp, w->Pi, w->Px, w->Ap, w->Ai, w->Ax, w->set.sigma,
                     w->rho_inv_vec);
    reset_info(w);
    return e;
}

/* osqp_update_settings as osqp-python 0.6 exposes it (update_max_iter, update_eps_abs, ...,
 * update_rho): the settings OSQP lets change after setup are copied; rho goes through
 * osqp_update_rho (clipped, rho vector by row class, KKT refactored).  sigma, scaling and
 * the adaptive-rho settings are fixed at setup: a different value is a validation error.
 * set_rho: only when the caller passes rho (osqp-python calls update_rho only then), so the
 * rho a previous solve adapted to stays otherwise. */
static int osqp_update_rho(orc_work *w, double rho_new);

int orc_update_settings(orc_work *w, const orc_settings *s, int set_rho) {
    const orc_settings *o = &w->set;
    if (s->sigma != o->sigma || s->scaling != o->scaling || s->adaptive_rho != o->adaptive_rho ||
        s->adaptive_rho_tolerance != o->adaptive_rho_tolerance ||
        (s->adaptive_rho_interval && s->adaptive_rho_interval != o->adaptive_rho_interval))
        return ORC_SETTINGS_VALIDATION_ERROR;
    if (s->max_iter <= 0 || s->eps_abs < 0 || s->eps_rel < 0 || (s->eps_abs == 0 && s->eps_rel == 0) ||
        s->eps_prim_inf <= 0 || s->eps_dual_inf <= 0 || s->alpha <= 0 || s->alpha >= 2 ||
        s->check_termination < 0 || s->rho <= 0 || s->delta <= 0 || s->polish_refine_iter < 0)
        return ORC_SETTINGS_VALIDATION_ERROR;
    const double rho = s->rho;
    w->set.max_iter = s->max_iter;
    w->set.eps_abs = s->eps_abs;
    w->set.eps_rel = s->eps_rel;
    w->set.eps_prim_inf = s->eps_prim_inf;
    w->set.eps_dual_inf = s->eps_dual_inf;
    w->set.alpha = s->alpha;
    w->set.delta = s->delta;
    w->set.polish = s->polish;
    w->set.polish_refine_iter = s->polish_refine_iter;
    w->set.scaled_termination = s->scaled_termination;
    w->set.check_termination = s->check_termination;
    w->set.warm_start = s->warm_start;
    if (set_rho && osqp_update_rho(w, rho)) return ORC_NONCVX_ERROR;
    return 0;
}

/* ---- auxil.c ---- */
static void swap_vectors(double **a, double **b) { double *t = *a; *a = *b; *b = t; }

static void cold_start(orc_work *w) {
    memset(w->x, 0, sizeof(double) * w->n);
    memset(w->z, 0, sizeof(double) * w->m);
    memset(w->y, 0, sizeof(double) * w->m);
}

static void update_xz_tilde(orc_work *w) {
    int n = w->n, m = w->m;
    for (int i = 0; i < n; ++i) w->xz_tilde[i] = w->set.sigma * w->x_prev[i] - w->q[i];
    for (int i = 0; i < m; ++i) w->xz_tilde[n + i] = w->z_prev[i] - w->rho_inv_vec[i] * w->y[i];
    /* solve_linsys_qdldl: sol = K \ b ; x_tilde = sol_x ; z_tilde = b_z + rho_inv .* nu */
    double *tmp = w->kkt->fw; /* free outside ldl_numeric; kkt_solve works in bp */
    memcpy(tmp, w->xz_tilde, sizeof(double) * (n + m));
    kkt_solve(w->kkt, tmp);
    for (int j = 0; j < n; ++j) w->xz_tilde[j] = tmp[j];
    for (int j = 0; j < m; ++j) w->xz_tilde[n + j] += w->rho_inv_vec[j] * tmp[n + j];
}

static void update_x(orc_work *w) {
    double a = w->set.alpha;
    for (int i = 0; i < w->n; ++i) w->x[i] = a * w->xz_tilde[i] + (1.0 - a) * w->x_prev[i];
    for (int i = 0; i < w->n; ++i) w->delta_x[i] = w->x[i] - w->x_prev[i];
}

static void update_z(orc_work *w) {
    double a = w->set.alpha;
    int n = w->n;
    for (int i = 0; i < w->m; ++i) {
        double v = a * w->xz_tilde[i + n] + (1.0 - a) * w->z_prev[i] + w->rho_inv_vec[i] * w->y[i];
        w->z[i] = dmin(dmax(v, w->l[i]), w->u[i]);
    }
}

static void update_y(orc_work *w) {
    double a = w->set.alpha;
    int n = w->n;
    for (int i = 0; i < w->m; ++i) {
        w->delta_y[i] = w->rho_vec[i] * (a * w->xz_tilde[i + n] + (1.0 - a) * w->z_prev[i] - w->z[i]);
        w->y[i] += w->delta_y[i];
    }
}

static double compute_obj_val(const orc_work *w, const double *x) {
    double r = quad_form(w, x);
    for (int j = 0; j < w->n; ++j) r += w->q[j] * x[j];
    if (w->set.scaling) r *= w->cinv;
    return r;
}

static double compute_pri_res(orc_work *w, const double *x, const double *z) {
    mat_vec(w->n, w->Ap, w->Ai, w->Ax, w->m, x, w->Axv, 0);
    for (int i = 0; i < w->m; ++i) w->z_prev[i] = w->Axv[i] - z[i];
    if (w->set.scaling && !w->set.scaled_termination)
        return vec_scaled_norm_inf(w->Einv, w->z_prev, w->m);
    return vec_norm_inf(w->z_prev, w->m);
}

static double compute_pri_tol(const orc_work *w, double eps_abs, double eps_rel) {
    double mx;
    if (w->set.scaling && !w->set.scaled_termination) {
        mx = vec_scaled_norm_inf(w->Einv, w->z, w->m);
        mx = dmax(mx, vec_scaled_norm_inf(w->Einv, w->Axv, w->m));
    } else {
        mx = dmax(vec_norm_inf(w->z, w->m), vec_norm_inf(w->Axv, w->m));
    }
    return eps_abs + eps_rel * mx;
}

static double compute_dua_res(orc_work *w, const double *x, const double *y) {
    int n = w->n;
    memcpy(w->x_prev, w->q, sizeof(double) * n);
    sym_mat_vec(w, x, w->Pxv);
    for (int j = 0; j < n; ++j) w->x_prev[j] += w->Pxv[j];
    if (w->m > 0) {
        mat_tpose_vec(n, w->Ap, w->Ai, w->Ax, y, w->Aty, 0, 0);
        for (int j = 0; j < n; ++j) w->x_prev[j] += w->Aty[j];
    }
    if (w->set.scaling && !w->set.scaled_termination)
        return w->cinv * vec_scaled_norm_inf(w->Dinv, w->x_prev, n);
    return vec_norm_inf(w->x_prev, n);
}

static double compute_dua_tol(const orc_work *w, double eps_abs, double eps_rel) {
    double mx;
    int n = w->n;
    if (w->set.scaling && !w->set.scaled_termination) {
        mx = vec_scaled_norm_inf(w->Dinv, w->q, n);
        mx = dmax(mx, vec_scaled_norm_inf(w->Dinv, w->Aty, n));
        mx = dmax(mx, vec_scaled_norm_inf(w->Dinv, w->Pxv, n));
        mx *= w->cinv;
    } else {
        mx = vec_norm_inf(w->q, n);
        mx = dmax(mx, vec_norm_inf(w->Aty, n));
        mx = dmax(mx, vec_norm_inf(w->Pxv, n));
    }
    return eps_abs + eps_rel * mx;
}

static int is_primal_infeasible(orc_work *w, double eps_prim_inf) {
    int m = w->m, n = w->n;
    double norm_dy, ineq_lhs = 0.0;
    for (int i = 0; i < m; ++i) {
        if (w->u[i] > OSQP_INFTY * MIN_SCALING) {
            if (w->l[i] < -OSQP_INFTY * MIN_SCALING) w->delta_y[i] = 0.0;
            else w->delta_y[i] = dmin(w->delta_y[i], 0.0);
        } else if (w->l[i] < -OSQP_INFTY * MIN_SCALING) {
            w->delta_y[i] = dmax(w->delta_y[i], 0.0);
        }
    }
    if (w->set.scaling && !w->set.scaled_termination) {
        for (int i = 0; i < m; ++i) w->Adelta_x[i] = w->E[i] * w->delta_y[i];
        norm_dy = vec_norm_inf(w->Adelta_x, m);
    } else {
        norm_dy = vec_norm_inf(w->delta_y, m);
    }
    if (norm_dy > eps_prim_inf) {
        for (int i = 0; i < m; ++i)
            ineq_lhs += w->u[i] * dmax(w->delta_y[i], 0.0) + w->l[i] * dmin(w->delta_y[i], 0.0);
        if (ineq_lhs < eps_prim_inf * norm_dy) {
            mat_tpose_vec(n, w->Ap, w->Ai, w->Ax, w->delta_y, w->Atdelta_y, 0, 0);
            if (w->set.scaling && !w->set.scaled_termination)
                for (int j = 0; j < n; ++j) w->Atdelta_y[j] *= w->Dinv[j];
            return vec_norm_inf(w->Atdelta_y, n) < eps_prim_inf * norm_dy;
        }
    }
    return 0;
}

static int is_dual_infeasible(orc_work *w, double eps_dual_inf) {
    int n = w->n, m = w->m;
    double norm_dx, cost_scaling;
    if (w->set.scaling && !w->set.scaled_termination) {
        norm_dx = vec_scaled_norm_inf(w->D, w->delta_x, n);
        cost_scaling = w->c;
    } else {
        norm_dx = vec_norm_inf(w->delta_x, n);
        cost_scaling = 1.0;
    }
    if (norm_dx > eps_dual_inf) {
        double qdx = 0.0;
        for (int j = 0; j < n; ++j) qdx += w->q[j] * w->delta_x[j];
        if (qdx < cost_scaling * eps_dual_inf * norm_dx) {
            sym_mat_vec(w, w->delta_x, w->Pdelta_x);
            if (w->set.scaling && !w->set.scaled_termination)
                for (int j = 0; j < n; ++j) w->Pdelta_x[j] *= w->Dinv[j];
            if (vec_norm_inf(w->Pdelta_x, n) < cost_scaling * eps_dual_inf * norm_dx) {
                mat_vec(n, w->Ap, w->Ai, w->Ax, m, w->delta_x, w->Adelta_x, 0);
                if (w->set.scaling && !w->set.scaled_termination)
                    for (int i = 0; i < m; ++i) w->Adelta_x[i] *= w->Einv[i];
                for (int i = 0; i < m; ++i) {
                    if ((w->u[i] < OSQP_INFTY * MIN_SCALING && w->Adelta_x[i] > eps_dual_inf * norm_dx) ||
                        (w->l[i] > -OSQP_INFTY * MIN_SCALING && w->Adelta_x[i] < -eps_dual_inf * norm_dx))
                        return 0;
                }
                return 1;
            }
        }
    }
    return 0;
}

static int check_termination(orc_work *w, int approximate) {
    double eps_abs = w->set.eps_abs, eps_rel = w->set.eps_rel;
    double eps_pinf = w->set.eps_prim_inf, eps_dinf = w->set.eps_dual_inf;
    int prim_ok = 0, dual_ok = 0, prim_inf = 0, dual_inf = 0;
    if (w->info.pri_res > OSQP_INFTY || w->info.dua_res > OSQP_INFTY) {
        w->info.status_val = ORC_NON_CVX;
        w->info.obj_val = NAN;
        return 1;
    }
    if (approximate) { eps_abs *= 10; eps_rel *= 10; eps_pinf *= 10; eps_dinf *= 10; }
    if (w->m == 0) {
        prim_ok = 1;
    } else {
        double ep = compute_pri_tol(w, eps_abs, eps_rel);
        if (w->info.pri_res < ep) prim_ok = 1;
        else prim_inf = is_primal_infeasible(w, eps_pinf);
    }
    double ed = compute_dua_tol(w, eps_abs, eps_rel);
    if (w->info.dua_res < ed) dual_ok = 1;
    else dual_inf = is_dual_infeasible(w, eps_dinf);

    if (prim_ok && dual_ok) {
        w->info.status_val = approximate ? ORC_SOLVED_INACCURATE : ORC_SOLVED;
        return 1;
    } else if (prim_inf) {
        w->info.status_val = approximate ? ORC_PRIMAL_INFEASIBLE_INACCURATE : ORC_PRIMAL_INFEASIBLE;
        if (w->set.scaling && !w->set.scaled_termination)
            for (int i = 0; i < w->m; ++i) w->delta_y[i] *= w->E[i];
        w->info.obj_val = OSQP_INFTY;
        return 1;
    } else if (dual_inf) {
        w->info.status_val = approximate ? ORC_DUAL_INFEASIBLE_INACCURATE : ORC_DUAL_INFEASIBLE;
        if (w->set.scaling && !w->set.scaled_termination)
            for (int j = 0; j < w->n; ++j) w->delta_x[j] *= w->D[j];
        w->info.obj_val = -OSQP_INFTY;
        return 1;
    }
    return 0;
}

static void update_info(orc_work *w, int iter, int compute_objective) {
    w->info.iter = iter;
    if (compute_objective) w->info.obj_val = compute_obj_val(w, w->x);
    if (w->m == 0) w->info.pri_res = 0.0;
    else w->info.pri_res = compute_pri_res(w, w->x, w->z);
    w->info.dua_res = compute_dua_res(w, w->x, w->y);
}

static double compute_rho_estimate(const orc_work *w) {
    int n = w->n, m = w->m;
    double pri = vec_norm_inf(w->z_prev, m);
    double dua = vec_norm_inf(w->x_prev, n);
    double pn = dmax(vec_norm_inf(w->z, m), vec_norm_inf(w->Axv, m));
    pri /= (pn + DIVISION_TOL);
    double dn = vec_norm_inf(w->q, n);
    dn = dmax(dn, vec_norm_inf(w->Aty, n));
    dn = dmax(dn, vec_norm_inf(w->Pxv, n));
    dua /= (dn + DIVISION_TOL);
    double r = w->set.rho * sqrt(pri / (dua + DIVISION_TOL));
    return dmin(dmax(r, RHO_MIN), RHO_MAX);
}

static int osqp_update_rho(orc_work *w, double rho_new) {
    if (rho_new <= 0) return -1;
    w->set.rho = dmin(dmax(rho_new, RHO_MIN), RHO_MAX);
    for (int i = 0; i < w->m; ++i) {
        if (w->constr_type[i] == 0) {
            w->rho_vec[i] = w->set.rho;
            w->rho_inv_vec[i] = 1.0 / w->set.rho;
        } else if (w->constr_type[i] == 1) {
            w->rho_vec[i] = RHO_EQ_OVER_RHO_INEQ * w->set.rho;
            w->rho_inv_vec[i] = 1.0 / w->rho_vec[i];
        }
    }
    return kkt_update_rho(w->kkt, w->rho_inv_vec);
}

static int adapt_rho(orc_work *w) {
    double rho_new = compute_rho_estimate(w);
    w->info.rho_estimate = rho_new;
    if (rho_new > w->set.rho * w->set.adaptive_rho_tolerance ||
        rho_new < w->set.rho / w->set.adaptive_rho_tolerance) {
        int e = osqp_update_rho(w, rho_new);
        w->info.rho_updates += 1;
        return e;
    }
    return 0;
}

static int has_solution(int st) {
    return st != ORC_PRIMAL_INFEASIBLE && st != ORC_PRIMAL_INFEASIBLE_INACCURATE &&
           st != ORC_DUAL_INFEASIBLE && st != ORC_DUAL_INFEASIBLE_INACCURATE && st != ORC_NON_CVX;
}

static void store_solution(orc_work *w) {
    int n = w->n, m = w->m;
    if (has_solution(w->info.status_val)) {
        memcpy(w->sol_x, w->x, sizeof(double) * n);
        memcpy(w->sol_y, w->y, sizeof(double) * m);
        if (w->set.scaling) {
            for (int j = 0; j < n; ++j) w->sol_x[j] *= w->D[j];
            for (int i = 0; i < m; ++i) { w->sol_y[i] *= w->E[i]; w->sol_y[i] *= w->cinv; }  /* unscale_solution */
        }
    } else {
        for (int j = 0; j < n; ++j) w->sol_x[j] = NAN;
        for (int i = 0; i < m; ++i) w->sol_y[i] = NAN;
        int st = w->info.status_val;
        if (st == ORC_PRIMAL_INFEASIBLE || st == ORC_PRIMAL_INFEASIBLE_INACCURATE) {
            double nv = vec_norm_inf(w->delta_y, m);
            for (int i = 0; i < m; ++i) w->delta_y[i] *= 1.0 / nv;
        }
        if (st == ORC_DUAL_INFEASIBLE || st == ORC_DUAL_INFEASIBLE_INACCURATE) {
            double nv = vec_norm_inf(w->delta_x, n);
            for (int j = 0; j < n; ++j) w->delta_x[j] *= 1.0 / nv;
        }
        cold_start(w);
    }
}

/* ---- polish.c (OSQP 0.6) restated ----
 * Guess the active constraints from the ADMM iterate (form_Ared), solve the
 * reduced KKT system [[P + delta I, Ared'], [Ared, -delta I]] [x; y_red] =
 * [-q; l_low; u_upp] with polish_refine_iter steps of iterative refinement against
 * the unregularised matrix, map y_red back, project (z, y) onto the normal cone,
 * and keep the polished point only if it lowers the residuals (or one of them is
 * already below 1e-10).  All on the scaled data, before store_solution. */
static void polish(orc_work *w) {
    int n = w->n, m = w->m;
    int *A_to_low = (int *)malloc(sizeof(int) * (m ? m : 1)), *A_to_upp = (int *)malloc(sizeof(int) * (m ? m : 1));
    int *low_to_A = (int *)malloc(sizeof(int) * (m ? m : 1)), *upp_to_A = (int *)malloc(sizeof(int) * (m ? m : 1));
    int n_low = 0, n_upp = 0;
    for (int j = 0; j < m; ++j) {
        if (w->z[j] - w->l[j] < -w->y[j]) { low_to_A[n_low] = j; A_to_low[j] = n_low++; }
        else A_to_low[j] = -1;
    }
    for (int j = 0; j < m; ++j) {
        if (w->u[j] - w->z[j] < w->y[j]) { upp_to_A[n_upp] = j; A_to_upp[j] = n_upp++; }
        else A_to_upp[j] = -1;
    }
    int mred = n_low + n_upp;
    /* Ared (CSC, column by column: lower-active copy, then upper-active copy) */
    int nnz = 0;
    for (int p = 0; p < w->Ap[n]; ++p) nnz += (A_to_low[w->Ai[p]] >= 0) + (A_to_upp[w->Ai[p]] >= 0);
    int *Rp = (int *)calloc(n + 1, sizeof(int)), *Ri = (int *)malloc(sizeof(int) * (nnz ? nnz : 1));
    double *Rx = (double *)malloc(sizeof(double) * (nnz ? nnz : 1));
    int q_ = 0;
    for (int j = 0; j < n; ++j) {
        for (int p = w->Ap[j]; p < w->Ap[j + 1]; ++p) {
            int i = w->Ai[p];
            if (A_to_low[i] >= 0) { Ri[q_] = A_to_low[i]; Rx[q_++] = w->Ax[p]; }
            if (A_to_upp[i] >= 0) { Ri[q_] = A_to_upp[i] + n_low; Rx[q_++] = w->Ax[p]; }
        }
        Rp[j + 1] = q_;
    }
    double *dinv = dalloc(mred), *rhs = dalloc(n + mred), *sol = dalloc(n + mred), *r2 = dalloc(n + mred);
    for (int i = 0; i < mred; ++i) dinv[i] = w->set.delta;
    kkt_t *k = NULL;
    int e = kkt_init(&k, n, mred, w->Pp, w->Pi, w->Px, Rp, Ri, Rx, w->set.delta, dinv);
    if (e) {
        w->info.status_polish = -1;
    } else {
        for (int j = 0; j < n; ++j) rhs[j] = -w->q[j];
        for (int i = 0; i < n_low; ++i) rhs[n + i] = w->l[low_to_A[i]];
        for (int i = 0; i < n_upp; ++i) rhs[n + n_low + i] = w->u[upp_to_A[i]];
        memcpy(sol, rhs, sizeof(double) * (n + mred));
        kkt_solve(k, sol);
        for (int it = 0; it < w->set.polish_refine_iter; ++it) {
            /* r2 = rhs - [[P, Ared'], [Ared, 0]] sol */
            memcpy(r2, rhs, sizeof(double) * (n + mred));
            sym_mat_vec(w, sol, w->Pxv);
            for (int j = 0; j < n; ++j) r2[j] -= w->Pxv[j];
            for (int j = 0; j < n; ++j)
                for (int p = Rp[j]; p < Rp[j + 1]; ++p) {
                    r2[j] -= Rx[p] * sol[n + Ri[p]];
                    r2[n + Ri[p]] -= Rx[p] * sol[j];
                }
            kkt_solve(k, r2);
            for (int j = 0; j < n + mred; ++j) sol[j] += r2[j];
        }
        double *px = dalloc(n), *pz = dalloc(m), *py = dalloc(m);
        memcpy(px, sol, sizeof(double) * n);
        mat_vec(n, w->Ap, w->Ai, w->Ax, m, px, pz, 0);
        for (int j = 0; j < m; ++j) {
            if (mred == 0) py[j] = 0.0;
            else if (A_to_low[j] >= 0) py[j] = sol[n + A_to_low[j]];
            else if (A_to_upp[j] >= 0) py[j] = sol[n + n_low + A_to_upp[j]];
            else py[j] = 0.0;
        }
        for (int j = 0; j < m; ++j) {  /* project_normalcone */
            double t = pz[j] + py[j];
            pz[j] = dmin(dmax(t, w->l[j]), w->u[j]);
            py[j] = t - pz[j];
        }
        double pobj = compute_obj_val(w, px);
        double ppri = m == 0 ? 0.0 : compute_pri_res(w, px, pz);
        double pdua = compute_dua_res(w, px, py);
        int ok = (ppri < w->info.pri_res && pdua < w->info.dua_res) ||
                 (ppri < w->info.pri_res && w->info.dua_res < 1e-10) ||
                 (pdua < w->info.dua_res && w->info.pri_res < 1e-10);
        if (ok) {
            w->info.obj_val = pobj;
            w->info.pri_res = ppri;
            w->info.dua_res = pdua;
            w->info.status_polish = 1;
            memcpy(w->x, px, sizeof(double) * n);
            memcpy(w->z, pz, sizeof(double) * m);
            memcpy(w->y, py, sizeof(double) * m);
        } else {
            w->info.status_polish = -1;
        }
        free(px); free(pz); free(py);
        kkt_free(k);
    }
    free(dinv); free(rhs); free(sol); free(r2); free(Rp); free(Ri); free(Rx);
    free(A_to_low); free(A_to_upp); free(low_to_A); free(upp_to_A);
}

int orc_solve(orc_work *w) {
    int iter, can_check = 0;
    int compute_cost = 0; /* verbose off */
    if (!w->kkt) {  /* a matrix update whose refactorisation failed (orc_update_P_A) */
        w->info.status_val = ORC_NON_CVX;
        w->info.iter = 0;
        store_solution(w);
        return ORC_NONCVX_ERROR;
    }
    if (!w->set.warm_start) cold_start(w);
    for (iter = 1; iter <= w->set.max_iter; ++iter) {
        swap_vectors(&w->x, &w->x_prev);
        swap_vectors(&w->z, &w->z_prev);
        update_xz_tilde(w);
        update_x(w);
        update_z(w);
        update_y(w);
        can_check = w->set.check_termination && (iter % w->set.check_termination == 0);
        if (can_check) {
            update_info(w, iter, compute_cost);
            if (check_termination(w, 0)) break;
        }
        if (w->set.adaptive_rho && w->set.adaptive_rho_interval &&
            (iter % w->set.adaptive_rho_interval == 0)) {
            if (!can_check) update_info(w, iter, compute_cost);
            if (adapt_rho(w)) {
                w->info.status_val = ORC_NON_CVX; /* linear system failure */
                break;
            }
        }
    }
    if (!can_check) {
        update_info(w, iter - 1, compute_cost);
        check_termination(w, 0);
    }
    if (!compute_cost && has_solution(w->info.status_val))
        w->info.obj_val = compute_obj_val(w, w->x);
    if (w->info.status_val == ORC_UNSOLVED) {
        if (!check_termination(w, 1)) w->info.status_val = ORC_MAX_ITER_REACHED;
    }
    w->info.rho_estimate = compute_rho_estimate(w);
    w->info.status_polish = 0;
    if (w->set.polish && w->info.status_val == ORC_SOLVED) polish(w);
    store_solution(w);
    return 0;
}

void orc_get_solution(const orc_work *w, double *x, double *y, double *pc, double *dc) {
    if (x) memcpy(x, w->sol_x, sizeof(double) * w->n);
    if (y) memcpy(y, w->sol_y, sizeof(double) * w->m);
    if (pc) memcpy(pc, w->delta_y, sizeof(double) * w->m);
    if (dc) memcpy(dc, w->delta_x, sizeof(double) * w->n);
}
void orc_get_info(const orc_work *w, orc_info *info) { *info = w->info; }
int orc_kkt_nnz_L(const orc_work *w) { return w->kkt->Lp[w->kkt->N]; }

/* ---- batch helper (baseline / tests) ---- */
typedef struct {
    int b0, b1, n, m;
    const int *Pp, *Pi, *Ap, *Ai;
    const double *Px_b, *q_b, *Ax_b, *l_b, *u_b;
    const double *x0_b, *y0_b;
    const orc_settings *s;
    double *x_out, *y_out;
    int *status, *iters;
    int err;
    double t_setup, t_solve; /* thread-seconds in orc_setup (+ warm start) and in orc_solve */
} batch_job;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void *batch_worker(void *arg) {
    batch_job *j = (batch_job *)arg;
    int nnzP = j->Pp[j->n], nnzA = j->Ap[j->n];
    for (int b = j->b0; b < j->b1; ++b) {
        orc_work *w = NULL;
        const double t0 = now_s();
        int e = orc_setup(&w, j->n, j->m, j->Pp, j->Pi, j->Px_b + (size_t)b * nnzP,
                          j->q_b + (size_t)b * j->n, j->Ap, j->Ai, j->Ax_b + (size_t)b * nnzA,
                          j->l_b + (size_t)b * j->m, j->u_b + (size_t)b * j->m, j->s);
        if (e) {
            if (!j->err) j->err = e;
            if (j->status) j->status[b] = ORC_NON_CVX;
            continue;
        }
        if (j->x0_b && j->y0_b) orc_warm_start(w, j->x0_b + (size_t)b * j->n, j->y0_b + (size_t)b * j->m);
        const double t1 = now_s();
        orc_solve(w);
        j->t_setup += t1 - t0;
        j->t_solve += now_s() - t1;
        orc_get_solution(w, j->x_out ? j->x_out + (size_t)b * j->n : NULL,
                         j->y_out ? j->y_out + (size_t)b * j->m : NULL, NULL, NULL);
        if (j->status) j->status[b] = w->info.status_val;
        if (j->iters) j->iters[b] = w->info.iter;
        orc_cleanup(w);
    }
    return NULL;
}

int orc_solve_batch(int B, int n, int m, const int *Pp, const int *Pi, const double *Px_b,
                    const double *q_b, const int *Ap, const int *Ai, const double *Ax_b,
                    const double *l_b, const double *u_b, const orc_settings *s,
                    double *x_out, double *y_out, int *status, int *iters, int nthreads) {
    return orc_solve_batch_warm(B, n, m, Pp, Pi, Px_b, q_b, Ap, Ai, Ax_b, l_b, u_b, NULL, NULL, s, x_out, y_out,
                                status, iters, nthreads);
}

int orc_solve_batch_warm(int B, int n, int m, const int *Pp, const int *Pi, const double *Px_b,
                         const double *q_b, const int *Ap, const int *Ai, const double *Ax_b,
                         const double *l_b, const double *u_b, const double *x0_b, const double *y0_b,
                         const orc_settings *s, double *x_out, double *y_out, int *status, int *iters,
                         int nthreads) {
    return orc_solve_batch_timed(B, n, m, Pp, Pi, Px_b, q_b, Ap, Ai, Ax_b, l_b, u_b, x0_b, y0_b, s, x_out, y_out,
                                 status, iters, nthreads, NULL);
}

int orc_solve_batch_timed(int B, int n, int m, const int *Pp, const int *Pi, const double *Px_b,
                          const double *q_b, const int *Ap, const int *Ai, const double *Ax_b,
                          const double *l_b, const double *u_b, const double *x0_b, const double *y0_b,
                          const orc_settings *s, double *x_out, double *y_out, int *status, int *iters,
                          int nthreads, double *phase_s) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > B) nthreads = B > 0 ? B : 1;
    batch_job *jobs = (batch_job *)calloc(nthreads, sizeof(batch_job));
    pthread_t *th = (pthread_t *)calloc(nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; ++t) {
        batch_job *j = &jobs[t];
        j->b0 = (int)((long long)B * t / nthreads);
        j->b1 = (int)((long long)B * (t + 1) / nthreads);
        j->n = n; j->m = m; j->Pp = Pp; j->Pi = Pi; j->Ap = Ap; j->Ai = Ai;
        j->Px_b = Px_b; j->q_b = q_b; j->Ax_b = Ax_b; j->l_b = l_b; j->u_b = u_b; j->s = s;
        j->x0_b = x0_b; j->y0_b = y0_b;
        j->x_out = x_out; j->y_out = y_out; j->status = status; j->iters = iters;
    }
    if (nthreads == 1) {
        batch_worker(&jobs[0]);
    } else {
        for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
        for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    }
    int err = 0;
    if (phase_s) phase_s[0] = phase_s[1] = 0.0;
    for (int t = 0; t < nthreads; ++t) {
        if (jobs[t].err && !err) err = jobs[t].err;
        if (phase_s) { phase_s[0] += jobs[t].t_setup; phase_s[1] += jobs[t].t_solve; }
    }
    free(jobs); free(th);
    return err;
}
