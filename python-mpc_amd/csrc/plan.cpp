// plan.cpp -- symbolic analysis of the shared sparsity pattern (see plan.h).
#include "plan.h"

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <queue>

namespace mpcqp {

// The wide batch setup's register lists (setup_wide.h), built here once per plan: its LDS
// byte addresses (Pv at 0, Ac, Dt, Et after it, lds_setup_wide_bytes's layout), 16 bits each,
// two to a word, so the kernel's prologue loads each word coalesced instead of chasing
// gcol / grow / gpsym / acsc_v / a_c per instance (with csc_pos, the A values load in the
// user's order, coalesced, and land at their padded-CSC places in LDS).  Built where that kernel applies
// (kernels.hip::setup_rw_fits: its LDS stays below 64 KiB), empty elsewhere.
static void build_wide_lists(Plan& pl) {
    pl.wide_cg.clear(); pl.wide_pg.clear(); pl.wide_rg.clear(); pl.wide_as.clear(); pl.wide_ps.clear();
    const int m = pl.m, npad = pl.npad, nnzA = pl.nnzA, nnzP = pl.nnzP;
    if (npad > 1024 || m > 1024 || pl.p_k > 4 || pl.gather_k > 8 || nnzA > 3 * 1024 || nnzP > 1024) return;
    const unsigned abase = 8u * (unsigned)(nnzP + 1), dbase = abase + 8u * (unsigned)(nnzA + 1),
                   ebase = dbase + 8u * (unsigned)npad;
    auto pk = [](unsigned lo, unsigned hi) { return (int)(lo | hi << 16); };
    auto aad = [&](int g) { return abase + 8u * ((unsigned)g & 0xFFFFu); };
    pl.wide_cg.resize((size_t)4 * npad);
    pl.wide_pg.resize((size_t)2 * npad);
    for (int pc = 0; pc < npad; ++pc) {
        for (int k = 0; k < 4; ++k)
            pl.wide_cg[(size_t)k * npad + pc] = pk(aad(pl.gcol[(size_t)(2 * k) * npad + pc]),
                                                   aad(pl.gcol[(size_t)(2 * k + 1) * npad + pc]));
        for (int k = 0; k < 2; ++k)
            pl.wide_pg[(size_t)k * npad + pc] = pk(8u * ((unsigned)pl.gpsym[(size_t)(2 * k) * npad + pc] & 0xFFFFu),
                                                   8u * ((unsigned)pl.gpsym[(size_t)(2 * k + 1) * npad + pc] & 0xFFFFu));
    }
    pl.wide_rg.resize((size_t)4 * m);
    for (int r = 0; r < m; ++r)
        for (int k = 0; k < 4; ++k)
            pl.wide_rg[(size_t)k * m + r] = pk(aad(pl.grow[(size_t)(2 * k) * m + r]), aad(pl.grow[(size_t)(2 * k + 1) * m + r]));
    pl.wide_as.resize(nnzA);
    for (int e = 0; e < nnzA; ++e)
        pl.wide_as[e] = pk(ebase + 8u * (unsigned)pl.acsc_row[e], dbase + 8u * (unsigned)pl.a_c[pl.acsc_v[e]]);
    pl.wide_ps.resize(nnzP);
    for (int v = 0; v < nnzP; ++v) pl.wide_ps[v] = pk(dbase + 8u * (unsigned)pl.p_r[v], dbase + 8u * (unsigned)pl.p_c[v]);
}

namespace {

struct Graph {
    std::vector<std::vector<int>> adj;
};

// BFS from `s` restricted to unvisited-in-component vertices; returns levels.
std::vector<std::vector<int>> bfs_levels(const Graph& g, int s, std::vector<int>& mark, int stamp) {
    std::vector<std::vector<int>> levels;
    std::vector<int> cur{s};
    mark[s] = stamp;
    while (!cur.empty()) {
        levels.push_back(cur);
        std::vector<int> nxt;
        for (int v : cur) {
            // Cuthill-McKee flavour: visit neighbours by increasing degree
            std::vector<int> nb;
            for (int w : g.adj[v])
                if (mark[w] != stamp) { mark[w] = stamp; nb.push_back(w); }
            std::stable_sort(nb.begin(), nb.end(), [&](int a, int b) {
                return g.adj[a].size() < g.adj[b].size();
            });
            nxt.insert(nxt.end(), nb.begin(), nb.end());
        }
        cur.swap(nxt);
    }
    return levels;
}

// balanced four-block merge (build_plan's balance4: the caller's choice -- api.hip asks for it on
// every plain plan); MPCQP_BALANCE=0 / 1 overrides it
bool balance_blocks(bool balance4) {
    static const int ov = [] {
        const char* b = getenv("MPCQP_BALANCE");  // (diagnostic override)
        return b ? (b[0] != '0' ? 1 : 0) : -1;
    }();
    return ov < 0 ? balance4 : ov == 1;
}

}  // namespace

std::string build_plan(int n, int m, const int32_t* Pp, const int32_t* Pi, const int32_t* Ap,
                       const int32_t* Ai, Plan& pl, bool eliminate, bool balance4) {
    char buf[256];
    if (n <= 0 || m < 0) return "invalid dimensions";
    if (Pp[0] != 0 || Ap[0] != 0) return "CSC column pointers must start at 0";
    for (int j = 0; j < n; ++j) {
        if (Pp[j + 1] < Pp[j] || Ap[j + 1] < Ap[j]) return "CSC column pointers must be nondecreasing";
        for (int p = Pp[j]; p < Pp[j + 1]; ++p)
            if (Pi[p] < 0 || Pi[p] > j) return "P must be upper triangular";
        for (int p = Ap[j]; p < Ap[j + 1]; ++p)
            if (Ai[p] < 0 || Ai[p] >= m) return "A row index out of range";
    }
    pl = Plan();
    pl.n = n; pl.m = m; pl.nnzP = Pp[n]; pl.nnzA = Ap[n];

    // rows of A
    std::vector<std::vector<std::pair<int, int>>> rows(m);  // (col, value idx)
    for (int j = 0; j < n; ++j)
        for (int p = Ap[j]; p < Ap[j + 1]; ++p) rows[Ai[p]].push_back({j, p});

    // graph of K = P + A'A (off-diagonal pattern)
    Graph g;
    g.adj.assign(n, {});
    for (int j = 0; j < n; ++j)
        for (int p = Pp[j]; p < Pp[j + 1]; ++p) {
            int i = Pi[p];
            if (i != j) { g.adj[i].push_back(j); g.adj[j].push_back(i); }
        }
    for (int r = 0; r < m; ++r)
        for (auto& a : rows[r])
            for (auto& b : rows[r])
                if (a.first != b.first) g.adj[a.first].push_back(b.first);
    for (auto& v : g.adj) {
        std::sort(v.begin(), v.end());
        v.erase(std::unique(v.begin(), v.end()), v.end());
    }

    // eliminated variables (Plan::eown): isolated vertices, and leaves whose neighbour keeps
    // a degree >= 2 (of a two-vertex component the higher index goes), at most one leaf per
    // parent, each with at most two A nonzeros (the four-wave kernel's rhs list, LE)
    std::vector<int> par(n, -2);  // -2: kept, -1: eliminated isolated, >= 0: eliminated leaf of par
    if (eliminate) {
        std::vector<char> has_leaf(n, 0);
        for (int j = 0; j < n; ++j) {
            if (Ap[j + 1] - Ap[j] > 2) continue;
            const size_t d = g.adj[j].size();
            if (d == 0) { par[j] = -1; continue; }
            if (d != 1) continue;
            const int p = g.adj[j][0];
            const size_t dp = g.adj[p].size();
            if ((dp >= 2 || j > p) && !has_leaf[p]) { par[j] = p; has_leaf[p] = 1; }
        }
        // the reduced graph: eliminated vertices dropped
        for (int j = 0; j < n; ++j)
            if (par[j] != -2) g.adj[j].clear();
        for (int v = 0; v < n; ++v) {
            auto& a = g.adj[v];
            a.erase(std::remove_if(a.begin(), a.end(), [&](int w) { return par[w] != -2; }), a.end());
        }
    }
    auto kept = [&](int v) { return par[v] == -2; };

    // components, pseudo-peripheral BFS level structures
    std::vector<int> comp(n, -1), mark(n, -1);
    std::vector<std::vector<int>> all_levels, iso_levels;
    int stamp = 0;
    for (int v0 = 0; v0 < n; ++v0) {
        if (comp[v0] >= 0 || !kept(v0)) continue;
        // collect component
        std::vector<int> cv{v0};
        comp[v0] = v0;
        for (size_t t = 0; t < cv.size(); ++t)
            for (int w : g.adj[cv[t]])
                if (comp[w] < 0) { comp[w] = v0; cv.push_back(w); }
        if (cv.size() == 1) { iso_levels.push_back({v0}); continue; }
        int s = cv[0];
        for (int v : cv)
            if (g.adj[v].size() < g.adj[s].size()) s = v;
        auto lv = bfs_levels(g, s, mark, stamp++);
        for (int it = 0; it < 16; ++it) {  // George-Liu pseudo-peripheral search
            int cand = lv.back()[0];
            for (int v : lv.back())
                if (g.adj[v].size() < g.adj[cand].size()) cand = v;
            auto lv2 = bfs_levels(g, cand, mark, stamp++);
            if (lv2.size() > lv.size()) { lv.swap(lv2); s = cand; }
            else {
                // prefer the narrower structure among equal-depth ones
                size_t w1 = 0, w2 = 0;
                for (auto& L : lv) w1 = std::max(w1, L.size());
                for (auto& L : lv2) w2 = std::max(w2, L.size());
                if (lv2.size() == lv.size() && w2 < w1) lv.swap(lv2);
                break;
            }
        }
        for (auto& L : lv) all_levels.push_back(L);
    }
    for (auto& L : iso_levels) all_levels.push_back(L);

    // merge consecutive levels into blocks of <= kS
    std::vector<std::vector<int>> blocks;
    for (auto& L : all_levels) {
        pl.max_level = std::max<int>(pl.max_level, (int)L.size());
        if ((int)L.size() > kS) {
            snprintf(buf, sizeof buf,
                     "unsupported sparsity: a level set of K has %zu > %d variables", L.size(), kS);
            return buf;
        }
        if (!blocks.empty() && blocks.back().size() + L.size() <= (size_t)kS)
            blocks.back().insert(blocks.back().end(), L.begin(), L.end());
        else
            blocks.push_back(L);
    }
    if (!eliminate && blocks.size() == 4 && balance_blocks(balance4)) {
        // balanced merge: the smallest block capacity that still merges the levels into four
        // blocks (cfg 2: 31 / 30 / 30 / 13 -> 26 / 25 / 25 / 28).  Levels stay whole: the blocks
        // stay block-tridiagonal with the same coupling rows at each block's top.  The four-wave
        // factorisation's stage 1 pre-pivots block 0 whole and the others past their coupling
        // rows, one wave each, so its critical path is max(bsize_0, bsize_k - amax): 31 -> 26
        // pivots on cfg 2 (factorisation 43.5 k -> 42.1 k cycles, the cfg-2 kernel 0.4308 ->
        // 0.4290 ms, same-box A/B of five runs each); it also keeps every block
        // within the dense-inverse form's static column counts (experimental build, DK).
        size_t tot = 0;
        for (auto& L : all_levels) tot += L.size();
        for (size_t cap = (tot + 3) / 4; cap < (size_t)kS; ++cap) {
            std::vector<std::vector<int>> b2;
            for (auto& L : all_levels) {
                if (!b2.empty() && b2.back().size() + L.size() <= cap) b2.back().insert(b2.back().end(), L.begin(), L.end());
                else b2.push_back(L);
            }
            bool fit = b2.size() == 4;
            for (auto& B : b2) fit = fit && B.size() <= cap;
            if (fit) { blocks.swap(b2); break; }
        }
    }
    if (eliminate) {
        // greedy packing: consecutive runs of kS variables of the level order, a level split
        // between two blocks.  Block-tridiagonal as long as no edge spans more than one block
        // boundary (checked); taken when it saves a block (reduced slack layout: 125 variables
        // in 4 blocks instead of 5 -- the four-wave kernel's shape)
        std::vector<int> order;
        for (auto& L : all_levels) order.insert(order.end(), L.begin(), L.end());
        const int nbg = ((int)order.size() + kS - 1) / kS;
        if (nbg < (int)blocks.size()) {
            std::vector<int> bof(n, -1);
            for (size_t t = 0; t < order.size(); ++t) bof[order[t]] = (int)t / kS;
            bool ok = true;
            for (int v : order)
                for (int w : g.adj[v]) ok = ok && std::abs(bof[v] - bof[w]) <= 1;
            if (ok) {
                blocks.assign(nbg, {});
                for (size_t t = 0; t < order.size(); ++t) blocks[t / kS].push_back(order[t]);
            }
        }
    }
    pl.nb = (int)blocks.size();
    pl.nbp = pl.nb * kS;
    pl.bsize.resize(pl.nb);
    pl.var_pad.assign(n, -1);
    for (int k = 0; k < pl.nb; ++k) {
        pl.bsize[k] = (int)blocks[k].size();
        for (int t = 0; t < pl.bsize[k]; ++t) pl.var_pad[blocks[k][t]] = k * kS + t;
    }
    // eliminated columns: owners (the parent's block column; isolated ones on free block
    // columns, lowest first), padded indices nbp + e in owner order
    pl.eown.assign(pl.nbp, -1);
    std::vector<int> owner_var(pl.nbp, -1);  // block column -> eliminated variable
    if (eliminate) {
        std::vector<int> iso;
        for (int j = 0; j < n; ++j) {
            if (par[j] >= 0) owner_var[pl.var_pad[par[j]]] = j;
            else if (par[j] == -1) iso.push_back(j);
        }
        size_t next = 0;
        for (int pc = 0; pc < pl.nbp && next < iso.size(); ++pc)
            if (owner_var[pc] < 0) owner_var[pc] = iso[next++];
        if (next < iso.size()) return build_plan(n, m, Pp, Pi, Ap, Ai, pl, false, balance4);  // no free columns left
        for (int pc = 0; pc < pl.nbp; ++pc)
            if (owner_var[pc] >= 0) {
                pl.eown[pc] = pl.nbp + pl.ne;
                pl.var_pad[owner_var[pc]] = pl.nbp + pl.ne++;
            }
    }
    pl.npad = pl.nbp + ((pl.ne + 1) & ~1);  // even: the arrays after a padded-column vector stay 16-byte aligned
    pl.pad_var.assign(pl.npad, -1);
    for (int j = 0; j < n; ++j) {
        if (pl.var_pad[j] < 0) return "internal: unplaced variable";
        pl.pad_var[pl.var_pad[j]] = j;
    }

    // A by padded column
    pl.acsc_ptr.assign(pl.npad + 1, 0);
    for (int pc = 0; pc < pl.npad; ++pc) {
        int j = pl.pad_var[pc];
        pl.acsc_ptr[pc + 1] = pl.acsc_ptr[pc] + (j >= 0 ? Ap[j + 1] - Ap[j] : 0);
    }
    pl.acsc_row.resize(pl.nnzA);
    pl.acsc_v.resize(pl.nnzA);
    for (int pc = 0; pc < pl.npad; ++pc) {
        int j = pl.pad_var[pc];
        if (j < 0) continue;
        int q = pl.acsc_ptr[pc];
        for (int p = Ap[j]; p < Ap[j + 1]; ++p, ++q) { pl.acsc_row[q] = Ai[p]; pl.acsc_v[q] = p; }
    }
    // A by row
    pl.acsr_ptr.assign(m + 1, 0);
    for (int r = 0; r < m; ++r) pl.acsr_ptr[r + 1] = pl.acsr_ptr[r] + (int)rows[r].size();
    pl.acsr_col.resize(pl.nnzA);
    pl.acsr_v.resize(pl.nnzA);
    for (int r = 0; r < m; ++r) {
        int q = pl.acsr_ptr[r];
        for (auto& e : rows[r]) { pl.acsr_col[q] = pl.var_pad[e.first]; pl.acsr_v[q] = e.second; ++q; }
    }
    for (int pc = 0; pc < pl.npad; ++pc) pl.max_col_nnz = std::max(pl.max_col_nnz, pl.acsc_ptr[pc + 1] - pl.acsc_ptr[pc]);
    for (int r = 0; r < m; ++r) pl.max_row_nnz = std::max(pl.max_row_nnz, pl.acsr_ptr[r + 1] - pl.acsr_ptr[r]);
    // full symmetric P by padded row
    std::vector<std::vector<std::pair<int, int>>> prow(pl.npad);
    pl.p_r.resize(pl.nnzP);
    pl.p_c.resize(pl.nnzP);
    for (int j = 0; j < n; ++j)
        for (int p = Pp[j]; p < Pp[j + 1]; ++p) {
            int i = Pi[p];
            int pi = pl.var_pad[i], pj = pl.var_pad[j];
            pl.p_r[p] = pi; pl.p_c[p] = pj;
            prow[pi].push_back({pj, p});
            if (i != j) prow[pj].push_back({pi, p});
        }
    pl.psym_ptr.assign(pl.npad + 1, 0);
    for (int r = 0; r < pl.npad; ++r) pl.psym_ptr[r + 1] = pl.psym_ptr[r] + (int)prow[r].size();
    for (int r = 0; r < pl.npad; ++r)
        for (auto& e : prow[r]) { pl.psym_col.push_back(e.first); pl.psym_v.push_back(e.second); }
    pl.a_r.resize(pl.nnzA);
    pl.a_c.resize(pl.nnzA);
    for (int j = 0; j < n; ++j)
        for (int p = Ap[j]; p < Ap[j + 1]; ++p) { pl.a_r[p] = Ai[p]; pl.a_c[p] = pl.var_pad[j]; }

    // assembly terms: key = block*2*S*S + tile index
    struct Term { long key; int a, b, r; };
    std::vector<Term> terms;
    const long SS = (long)kS * kS;
    std::string err;
    auto add = [&](int pi, int pj, int a, int b, int r) {
        if (pi >= pl.nbp || pj >= pl.nbp) return;  // an eliminated column: its terms are etterm's
        int bi = pi / kS, bj = pj / kS, li = pi % kS, lj = pj % kS;
        if (bi == bj) terms.push_back({bi * 2 * SS + li * kS + lj, a, b, r});
        else if (bi == bj + 1) terms.push_back({bi * 2 * SS + SS + li * kS + lj, a, b, r});
        else if (bj == bi + 1) { /* upper block: covered by the transposed entry */ }
        else err = "internal: coupling beyond neighbouring blocks";
    };
    for (int r = 0; r < pl.npad; ++r)
        for (auto& e : prow[r]) add(r, e.first, e.second, 0, -1);
    for (int r = 0; r < m; ++r)
        for (auto& a : rows[r])
            for (auto& b : rows[r]) add(pl.var_pad[a.first], pl.var_pad[b.first], a.second, b.second, r);
    if (!err.empty()) return err;
    std::stable_sort(terms.begin(), terms.end(), [](const Term& x, const Term& y) { return x.key < y.key; });
    pl.asm_blk_ptr.assign(pl.nb + 1, 0);
    pl.asm_term_ptr.push_back(0);
    for (size_t t = 0; t < terms.size();) {
        size_t u = t;
        while (u < terms.size() && terms[u].key == terms[t].key) {
            pl.term_a.push_back(terms[u].a);
            pl.term_b.push_back(terms[u].b);
            pl.term_r.push_back(terms[u].r);
            ++u;
        }
        int blk = (int)(terms[t].key / (2 * SS));
        pl.asm_tgt.push_back((int)(terms[t].key % (2 * SS)));
        pl.asm_term_ptr.push_back((int)pl.term_a.size());
        pl.asm_blk_ptr[blk + 1]++;
        t = u;
    }
    for (int k = 0; k < pl.nb; ++k) pl.asm_blk_ptr[k + 1] += pl.asm_blk_ptr[k];
    // within a block, targets by descending term count (stable): the kernels' assembly
    // loops run a wave's targets for the count of its first one (tcnt), not term_max
    // (cfg 2: 720 of 984 targets have a single term, term_max is 6).  Each target's terms
    // keep their order, so the sums are unchanged.
    {
        std::vector<int> tg2, tp2{0}, ta2, tb2, tr2;
        for (int k = 0; k < pl.nb; ++k) {
            std::vector<int> ord;
            for (int t = pl.asm_blk_ptr[k]; t < pl.asm_blk_ptr[k + 1]; ++t) ord.push_back(t);
            auto cnt = [&](int t) { return pl.asm_term_ptr[t + 1] - pl.asm_term_ptr[t]; };
            std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return cnt(x) > cnt(y); });
            for (int t : ord) {
                tg2.push_back(pl.asm_tgt[t]);
                for (int u = pl.asm_term_ptr[t]; u < pl.asm_term_ptr[t + 1]; ++u) {
                    ta2.push_back(pl.term_a[u]); tb2.push_back(pl.term_b[u]); tr2.push_back(pl.term_r[u]);
                }
                tp2.push_back((int)ta2.size());
            }
        }
        pl.asm_tgt.swap(tg2); pl.asm_term_ptr.swap(tp2);
        pl.term_a.swap(ta2); pl.term_b.swap(tb2); pl.term_r.swap(tr2);
    }
    // A-pair terms address A values by their position in the padded-CSC order
    // (the order the solve kernel keeps them in LDS)
    std::vector<int> csc_pos(pl.nnzA);
    for (int e = 0; e < pl.nnzA; ++e) csc_pos[pl.acsc_v[e]] = e;
    for (size_t t = 0; t < pl.term_a.size(); ++t)
        if (pl.term_r[t] >= 0) { pl.term_a[t] = csc_pos[pl.term_a[t]]; pl.term_b[t] = csc_pos[pl.term_b[t]]; }
    // terms in ELL order: slot j of target t at (j * ntgt + t), two ints each:
    // (a | b << 16, r) for an A pair, (a | 0, -1) for a P value, zero padding
    // (nnzA | nnzA << 16, 0) -- Acsc[nnzA] is the kernels' zero slot
    pl.ntgt = (int)pl.asm_tgt.size();
    pl.term_max = 0;
    pl.tcnt.resize(pl.ntgt);
    for (int t = 0; t < pl.ntgt; ++t) {
        pl.tcnt[t] = pl.asm_term_ptr[t + 1] - pl.asm_term_ptr[t];
        pl.term_max = std::max(pl.term_max, pl.tcnt[t]);
    }
    pl.tterm.assign((size_t)2 * pl.ntgt * pl.term_max, 0);
    for (int t = 0; t < pl.ntgt; ++t)
        for (int j = 0; j < pl.term_max; ++j) {
            const int u = pl.asm_term_ptr[t] + j;
            int* w = &pl.tterm[2 * ((size_t)j * pl.ntgt + t)];
            if (u < pl.asm_term_ptr[t + 1]) {
                w[0] = pl.term_a[u] | (pl.term_r[u] >= 0 ? pl.term_b[u] << 16 : 0);
                w[1] = pl.term_r[u];
            } else {
                w[0] = pl.nnzA | (pl.nnzA << 16);
                w[1] = 0;
            }
        }
    for (size_t t = 0; t < pl.asm_tgt.size(); ++t)
        if (pl.asm_tgt[t] >= SS) pl.amax = std::max(pl.amax, (int)((pl.asm_tgt[t] - SS) / kS) + 1);
    {
        std::vector<int> cmin(pl.nb, kS), cmax(pl.nb, -1);
        for (int k = 1; k < pl.nb; ++k)
            for (int t = pl.asm_blk_ptr[k]; t < pl.asm_blk_ptr[k + 1]; ++t)
                if (pl.asm_tgt[t] >= SS) {
                    const int c = (pl.asm_tgt[t] - (int)SS) % kS;
                    cmin[k - 1] = std::min(cmin[k - 1], c);
                    cmax[k - 1] = std::max(cmax[k - 1], c);
                }
        pl.bmax = 1;
        for (int k = 0; k < pl.nb; ++k)
            if (cmax[k] >= 0) pl.bmax = std::max(pl.bmax, cmax[k] - cmin[k] + 1);
        pl.toff.assign(pl.nb, 0);
        for (int k = 0; k < pl.nb; ++k) pl.toff[k] = cmax[k] >= 0 ? std::min(cmin[k], kS - pl.bmax) : 0;
    }
    pl.acsr_pos.resize(pl.nnzA);
    for (int e = 0; e < pl.nnzA; ++e) pl.acsr_pos[e] = csc_pos[pl.acsr_v[e]];
    pl.csc_pos = csc_pos;
    // eliminated columns: the terms of K_jj and K_pj (etterm)
    if (pl.ne) {
        auto pidx = [&](int i, int j) {  // value index of P(i, j) in the user's triu CSC, or -1
            const int r = std::min(i, j), c = std::max(i, j);
            for (int p = Pp[c]; p < Pp[c + 1]; ++p)
                if (Pi[p] == r) return p;
            return -1;
        };
        std::vector<std::vector<std::pair<int, int>>> et(2 * pl.ne);  // (a | b << 16, r)
        for (int pc = 0; pc < pl.nbp; ++pc) {
            if (pl.eown[pc] < 0) continue;
            const int e = pl.eown[pc] - pl.nbp, j = pl.pad_var[pl.eown[pc]], p = par[j];
            pl.ecnt = std::max(pl.ecnt, Ap[j + 1] - Ap[j]);
            if (int v = pidx(j, j); v >= 0) et[2 * e].push_back({v, -1});
            for (int q = Ap[j]; q < Ap[j + 1]; ++q) et[2 * e].push_back({csc_pos[q] | (csc_pos[q] << 16), Ai[q]});
            if (p < 0) continue;
            if (int v = pidx(p, j); v >= 0) et[2 * e + 1].push_back({v, -1});
            for (int q = Ap[j]; q < Ap[j + 1]; ++q)
                for (int qp = Ap[p]; qp < Ap[p + 1]; ++qp)
                    if (Ai[qp] == Ai[q]) et[2 * e + 1].push_back({csc_pos[qp] | (csc_pos[q] << 16), Ai[q]});
        }
        pl.eterm_max = 1;
        for (auto& t : et) pl.eterm_max = std::max(pl.eterm_max, (int)t.size());
        const int nt = 2 * pl.ne;
        pl.etterm.assign((size_t)2 * nt * pl.eterm_max, 0);
        for (int t = 0; t < nt; ++t)
            for (int k = 0; k < pl.eterm_max; ++k) {
                int* w = &pl.etterm[2 * ((size_t)k * nt + t)];
                if (k < (int)et[t].size()) { w[0] = et[t][k].first; w[1] = et[t][k].second; }
                else { w[0] = pl.nnzA | (pl.nnzA << 16); w[1] = 0; }
            }
    }
    // packed gather lists (16-bit value position | 16-bit vector index << 16), padded
    // to kGS entries with (nnzA | 0): position nnzA holds a zero in the kernels' LDS copy
    pl.gather_k = std::max(pl.max_col_nnz, pl.max_row_nnz);
    if (pl.gather_k > kGS) return "unsupported sparsity: a row or column of A has more than 16 nonzeros";
    if (pl.nnzA >= 65535 || m >= 65536 || pl.npad >= 65536) return "unsupported size: nnz(A), m and n must be < 65535";
    const int pad = pl.nnzA;
    pl.gcol.assign((size_t)pl.npad * kGS, pad);
    for (int pc = 0; pc < pl.npad; ++pc)
        for (int e = pl.acsc_ptr[pc], k = 0; e < pl.acsc_ptr[pc + 1]; ++e, ++k)
            pl.gcol[(size_t)k * pl.npad + pc] = e | (pl.acsc_row[e] << 16);
    // P by padded column (full symmetric), padded with (nnzP | 0): Pv[nnzP] is a zero slot
    pl.p_k = 0;
    for (int r = 0; r < pl.npad; ++r) pl.p_k = std::max(pl.p_k, pl.psym_ptr[r + 1] - pl.psym_ptr[r]);
    if (pl.p_k > kGS) return "unsupported sparsity: a column of P has more than 16 nonzeros";
    if (pl.nnzP >= 65535) return "unsupported size: nnz(P) must be < 65535";
    pl.gpsym.assign((size_t)pl.npad * kGS, pl.nnzP);
    for (int r = 0; r < pl.npad; ++r)
        for (int e = pl.psym_ptr[r], k = 0; e < pl.psym_ptr[r + 1]; ++e, ++k)
            pl.gpsym[(size_t)k * pl.npad + r] = pl.psym_v[e] | (pl.psym_col[e] << 16);
    pl.grow.assign((size_t)m * kGS, pad);
    for (int r = 0; r < m; ++r)
        for (int e = pl.acsr_ptr[r], k = 0; e < pl.acsr_ptr[r + 1]; ++e, ++k)
            pl.grow[(size_t)k * m + r] = pl.acsr_pos[e] | (pl.acsr_col[e] << 16);
    build_wide_lists(pl);
    return "";
}

}  // namespace mpcqp
