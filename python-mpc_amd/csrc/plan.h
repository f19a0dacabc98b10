// plan.h -- host-side symbolic analysis for the MI355X batched QP solver.
//
// Everything here depends only on the SHARED sparsity pattern of the batch
// (P upper-triangular CSC, A CSC -- the arrays osqp.OSQP().setup() receives at
// vehicle_lateral_mpc_slack_increment.py:121 / Control/MPC/mpc_dynamics.py:393).
// It is computed once per handle; no per-instance numbers are touched on the
// host.
//
// The reduced KKT matrix  K = P + sigma I + A' diag(rho) A  (SPD, n x n) is
// put in block-tridiagonal form: breadth-first level sets of K's graph (per
// connected component, from a pseudo-peripheral vertex) only couple to the
// neighbouring level, so consecutive levels merged into blocks of <= S
// variables give  K = tridiag(E_k, D_k, E_{k+1}').  Every variable gets a
// "padded" index  k*S + local  so the device works on uniform S x S tiles.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace mpcqp {

constexpr int kS = 32;  // block (tile) size
constexpr int kGS = 16; // gather-list stride (max nonzeros per row / column of A)

struct Plan {
    int n = 0, m = 0, nb = 0, npad = 0, nnzP = 0, nnzA = 0;
    std::vector<int> bsize;       // [nb]
    std::vector<int> var_pad;     // [n]    user variable -> padded index
    std::vector<int> pad_var;     // [npad] padded index -> user variable or -1
    // A by padded column (CSC): entries (row, value index into user Ax)
    std::vector<int> acsc_ptr, acsc_row, acsc_v;
    // A by row (CSR): entries (padded column, value index)
    std::vector<int> acsr_ptr, acsr_col, acsr_v;
    // full symmetric P by padded row: (padded column, value index into user Px)
    std::vector<int> psym_ptr, psym_col, psym_v;
    // per stored value: padded row / column
    std::vector<int> p_r, p_c;    // [nnzP] (upper triangle of the user's P)
    std::vector<int> a_r, a_c;    // [nnzA] (row, padded column)
    // K assembly.  Per block k the device fills two S*S tiles:
    //   D_k (local index i*S+j)  and  E_k = K(block k, block k-1) (index S*S + i*S + j).
    // Targets of block k: asm_tgt[asm_blk_ptr[k] .. asm_blk_ptr[k+1]),
    // terms of target t: [asm_term_ptr[t], asm_term_ptr[t+1]).
    // term: r >= 0  -> rho[r] * Acsc[a] * Acsc[b] (positions in the padded-CSC order);
    //       r == -1 -> Px[a] (user order).
    std::vector<int> asm_blk_ptr, asm_tgt, asm_term_ptr, term_a, term_b, term_r;
    // the same terms, padded to term_max per target, in ELL order (see plan.cpp)
    int ntgt = 0, term_max = 0;
    std::vector<int> tterm;
    std::vector<int> tcnt;        // [ntgt] terms of each target (descending within a block)
    std::vector<int> csc_pos;     // [nnzA] user value index -> padded-CSC position
    std::vector<int> acsr_pos;    // [nnzA] CSR entry -> padded-CSC position of its value
    int max_level = 0;            // largest BFS level (diagnostic)
    int max_row_nnz = 0, max_col_nnz = 0;
    int gather_k = 0;             // max(max_row_nnz, max_col_nnz)
    // packed gather lists: [kGS][npad] by padded column (A' w), [kGS][m] by row (A x):
    // (position of the value in the padded-CSC order) | (vector index << 16), padding (nnzA | 0).
    // Entry k of every column (row) is contiguous, so the kernels' per-lane list loads
    // (lane = column / row) are coalesced.
    std::vector<int> gcol, grow;
    int p_k = 0;                  // max nonzeros per column of the symmetric P
    std::vector<int> gpsym;       // [kGS][npad] P by padded column: (Pv index) | (padded column << 16)
    // the wide batch setup's lists (plan.cpp::build_wide_lists; empty where it does not apply):
    // LDS byte addresses two to a word -- [4][npad] A and [2][npad] P by column, [4][m] A by
    // row, [nnzA] (Et row | Dt column) per padded-CSC value, [nnzP] (Dt row | Dt column) per P
    // value -- and csc_pos, user A value index -> padded-CSC position
    std::vector<int> wide_cg, wide_pg, wide_rg, wide_as, wide_ps;
    int amax = 0;                 // max over k of (last nonzero local row of E_k) + 1: F_k rows / H_{k-1} cols
    // the other side of the coupling: the columns of E_{k+1} (variables of block k that
    // couple to block k+1, its last BFS level) lie in [toff[k], toff[k] + bmax)
    std::vector<int> toff;        // [nb]
    int bmax = 0;
    // Eliminated variables (build_plan's `eliminate`): vertices of K's graph with at most one
    // neighbour -- a leaf (the slack of a soft constraint couples only to the state it
    // relaxes, vehicle_lateral_mpc_slack_increment.py:104-110) or an isolated vertex (the
    // slack layout's dead u_prev slack columns) -- are taken out of the
    // block-tridiagonal system by a scalar Schur complement: K_pp -= K_pj^2 / K_jj on the
    // parent's diagonal, b_p -= (K_pj / K_jj) b_j on its right-hand side, and after the
    // reduced solve  x_j = (b_j - K_pj x_p) / K_jj  elementwise.  They get the padded
    // indices [nbp, nbp + ne) after the block columns (npad = nbp + ne, rounded up to
    // even); every other per-column structure (gather lists, P rows) covers them as usual.
    int nbp = 0;                  // block columns nb * S
    int ne = 0;                   // eliminated variables
    int ecnt = 0;                 // most A nonzeros in an eliminated column
    std::vector<int> eown;        // [nbp] block column -> the eliminated column it owns (parent, or a
                                  //       free column for an isolated one), -1: none
    // K_jj (target 2e) and K_pj (target 2e + 1) of eliminated column nbp + e as ELL terms in
    // tterm's format: slot j of target t at (j * 2 ne + t)
    int eterm_max = 0;
    std::vector<int> etterm;
    // Which plan a handle took (api.hip::choose_plan): 0 the plain plan (elimination not
    // tried: polish, MPCQP_ELIM=0, an MPCQP_VARIANT override), 1 the eliminated plan, 2 an
    // eliminated plan was built but the four-wave kernel's shape did not fit it (choice_note
    // says which precondition failed), 3 nothing to eliminate
    int choice = 0;
    std::string choice_note;
    // identity of the plan's contents (api.hip: a fresh value per build, kept by the plan cache's
    // copies), so that a pooled device copy of the same plan is reused without an upload
    unsigned long long uid = 0;
};

// Returns "" on success, otherwise an error message.  eliminate: take degree <= 1
// vertices of K's graph out of the block system (see Plan::eown); the blocks are then
// packed greedily (consecutive runs of S variables of the level order) when that gives
// fewer blocks and stays block-tridiagonal.  balance4: a plain plan of four blocks is merged
// into four balanced ones (the experimental dense-inverse form, solve_wave.hip::dense_w4_on).
std::string build_plan(int n, int m, const int32_t* Pp, const int32_t* Pi,
                       const int32_t* Ap, const int32_t* Ai, Plan& out, bool eliminate = false,
                       bool balance4 = false);

}  // namespace mpcqp
