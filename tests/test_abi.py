"""Host-side checks of the C-ABI library (no GPU needed).

* libmpcqp.so loads and exports every function include/mpcqp.h declares;
* default settings are OSQP 0.6's (settings in force);
* the symbolic plan (mpcqp_analyze) puts K = P + sigma I + A' diag(rho) A into
  block-tridiagonal form with blocks <= the tile size, for every reference layout;
* argument / settings / sparsity validation raise the osqp-python exception
  types before any device is touched, and without a GPU the solver refuses to
  run (no CPU fallback).
"""
import ctypes as C
import json
import os
import re
import subprocess
import sys

import numpy as np
import pytest
import scipy.sparse as sparse

import osqp_amd
from osqp_amd import mpc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mpcqp.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mpcqp_\w+)\s*\(", text)))


def test_library_exports_header_symbols():
    names = header_functions()
    assert len(names) >= 20
    lib = C.CDLL(osqp_amd.LIB_PATH)
    missing = [nm for nm in names if not hasattr(lib, nm)]
    assert not missing, missing


def test_default_settings_are_osqp_06():
    s = osqp_amd._Settings()
    osqp_amd.lib().mpcqp_default_settings(C.byref(s))
    assert (s.rho, s.sigma, s.alpha) == (0.1, 1e-6, 1.6)
    assert (s.eps_abs, s.eps_rel, s.eps_prim_inf, s.eps_dual_inf) == (1e-3, 1e-3, 1e-4, 1e-4)
    assert (s.max_iter, s.scaling, s.check_termination, s.warm_start) == (4000, 10, 25, 1)
    assert (s.adaptive_rho, s.adaptive_rho_tolerance, s.polish) == (1, 5.0, 0)
    assert (s.delta, s.polish_refine_iter) == (1e-6, 3)


def _kkt_pattern(P, A):
    P = sparse.csc_matrix(P)
    A = sparse.csc_matrix(A)
    K = (abs(P) + abs(P).T + abs(A).T @ abs(A)).tocoo()
    return K.row, K.col


@pytest.mark.parametrize("cfg", [1, 2, 3, 5])
def test_plan_is_block_tridiagonal(cfg):
    b = mpc.make_batch(cfg, B=2, seed=3)
    P, _ = osqp_amd._drop_common_zeros(b["P"], b["Px"])
    A, _ = osqp_amd._drop_common_zeros(b["A"], b["Ax"])
    nb, blk, var_pad, bsize = osqp_amd.analyze(P, A)
    n = P.shape[0]
    assert blk == 32 and nb >= 1
    assert np.all(bsize >= 1) and np.all(bsize <= blk)
    assert len(np.unique(var_pad)) == n and var_pad.min() >= 0 and var_pad.max() < nb * blk
    block = var_pad // blk
    assert np.all(np.bincount(block, minlength=nb) == bsize)
    r, c = _kkt_pattern(P, A)
    assert np.max(np.abs(block[r] - block[c])) <= 1


@pytest.mark.parametrize("name", ["slack_n20", "vanilla_n20", "dyn_incr_n50", "kin_incr_n40"])
def test_plan_on_reference_fixtures(golden, name):
    g = golden(name + ".npz")
    P, A = g["P"], g["A"]
    nb, blk, var_pad, bsize = osqp_amd.analyze(P, A)
    block = var_pad // blk
    r, c = _kkt_pattern(osqp_amd.canonical_data(P, A)[0], A)
    assert np.max(np.abs(block[r] - block[c])) <= 1
    assert bsize.sum() == P.shape[0]


def test_dense_row_is_unsupported():
    n = 20
    P = sparse.eye(n, format="csc")
    A = sparse.csc_matrix(np.ones((1, n)))  # one row with 20 > 16 nonzeros
    with pytest.raises(NotImplementedError):
        osqp_amd.analyze(P, A)


def _tiny():
    P = sparse.diags([2.0, 1.0], format="csc")
    A = sparse.csc_matrix(np.array([[1.0, 1.0], [1.0, 0.0], [0.0, 1.0]]))
    return P, np.array([1.0, 1.0]), A, np.array([1.0, 0.0, 0.0]), np.array([1.0, 0.7, 0.7])


def test_setup_validation_errors():
    P, q, A, l, u = _tiny()
    with pytest.raises(ValueError):
        osqp_amd.OSQP().setup(P, q, A, l, u, alpha=2.5)
    with pytest.raises(ValueError):
        osqp_amd.OSQP().setup(P, q, A, l, u, max_iter=0)
    with pytest.raises(ValueError):
        osqp_amd.OSQP().setup(P, q[:1], A, l, u)
    with pytest.raises(ValueError):
        osqp_amd.OSQP().setup(P, q, A, l, u, polish=True, delta=-1.0)
    with pytest.raises(ValueError):
        osqp_amd.OSQP().setup(P, q, A, l, u, polish=True, polish_refine_iter=-1)


def test_no_cpu_fallback_without_device():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    P, q, A, l, u = _tiny()
    with pytest.raises(RuntimeError, match="no HIP device"):
        osqp_amd.OSQP().setup(P, q, A, l, u, verbose=False)


@pytest.mark.parametrize("cfg", [1, 3])
def test_elimination_plan_slack_layout(cfg):
    """The plan the four-wave kernel runs for the slack layouts (plan.h Plan::eown): the 84
    live slack columns (leaves of K's graph: each touches only the state it relaxes) and
    the 21 dead u_prev slack columns (isolated) leave the block system, whose 125 variables
    then pack into 4 blocks of 32 (block-tridiagonal in the reduced graph)."""
    b = mpc.make_batch(cfg, B=2, seed=3)
    P, _ = osqp_amd._drop_common_zeros(b["P"], b["Px"])
    A, _ = osqp_amd._drop_common_zeros(b["A"], b["Ax"])
    nb, blk, var_pad, bsize, ne = osqp_amd.analyze(P, A, eliminate=True)
    n = P.shape[0]
    assert (n, nb, ne) == (230, 4, 105) and bsize.sum() == n - ne
    assert len(np.unique(var_pad)) == n
    elim = var_pad >= nb * blk
    assert elim.sum() == ne and np.all(elim[125:] == (np.arange(125, 230) >= 125))  # the slack block s_0..s_N
    r, c = _kkt_pattern(P, A)
    keep = ~elim[r] & ~elim[c]
    block = var_pad // blk
    assert np.max(np.abs(block[r[keep]] - block[c[keep]])) <= 1
    # each eliminated column couples to at most one kept column, never to another eliminated one
    off = r != c
    assert not np.any(elim[r[off]] & elim[c[off]])
    assert np.bincount(r[off & elim[r]], minlength=n).max() <= 1


@pytest.mark.parametrize("cfg,nb,amax_max,variant,choice,ne", [
    (1, 4, 8, 17, 1, 105),   # slack N = 20: the reduced system in the four-wave kernel
    (3, 4, 8, 17, 1, 105),
    (2, 4, 8, 17, 3, 0),     # vanilla N = 20: nothing to eliminate, four-wave kernel
    (5, 17, 16, 12, 3, 0),   # incremental dynamic N = 50: the long-horizon kernel
])
def test_plan_preview_pins_each_workloads_kernel(cfg, nb, amax_max, variant, choice, ne):
    """mpcqp_plan_preview (host only): the plan and kernel variant a handle would take.  The
    slack layouts' eliminated plan must keep amax <= 8 (the four-wave kernel's coupling rows);
    a regression in the level ordering or the greedy packing would otherwise fall back to
    the plain 8-block plan quietly (2x slower) -- here it fails, and plan_choice / note say
    why (plan.cpp greedy packing)."""
    b = mpc.make_batch(cfg, B=2, seed=3)
    P, _ = osqp_amd._drop_common_zeros(b["P"], b["Px"])
    A, _ = osqp_amd._drop_common_zeros(b["A"], b["Ax"])
    info = osqp_amd.plan_preview(P, A, **b["settings"])
    assert info["note"] == "", info["note"]
    assert (info["nb"], info["variant"], info["plan_choice"], info["n_eliminated"]) == (nb, variant, choice, ne)
    assert info["amax"] <= amax_max
    # polish factors the full system: the plain plan, elimination not tried
    pol = osqp_amd.plan_preview(P, A, **dict(b["settings"], polish=True))
    assert pol["plan_choice"] == 0 and pol["n_eliminated"] == 0


def test_balanced_four_block_merge():
    """The planner merges cfg 2's BFS levels into four balanced blocks (26 / 25 / 25 / 28 instead
    of the greedy 31 / 30 / 30 / 13: the four-wave factorisation's stage-1 critical path 31 -> 26
    pivots, and every block within the experimental dense-inverse form's static 26 / 28 columns
    per half) that stay block-tridiagonal with the same coupling rows -- in the production and
    the experimental build alike; MPCQP_BALANCE=0 (read once per process: a child) restores the
    greedy merge."""
    code = r"""
import json, sys
import numpy as np
import osqp_amd
from osqp_amd import mpc
b = mpc.make_batch(2, B=2, seed=3)
P, _ = osqp_amd._drop_common_zeros(b["P"], b["Px"])
A, _ = osqp_amd._drop_common_zeros(b["A"], b["Ax"])
nb, blk, var_pad, bsize = osqp_amd.analyze(P, A)
info = osqp_amd.plan_preview(P, A, **b["settings"])
K = (abs(P) + abs(P).T + abs(A).T @ abs(A)).tocoo()
blk_of = np.asarray(var_pad) // blk
span = int(np.abs(blk_of[K.row] - blk_of[K.col]).max())
print(json.dumps(dict(nb=int(nb), bsize=[int(v) for v in bsize], span=span, amax=info["amax"],
                      variant=info["variant"])))
"""
    env = dict(os.environ, MPCQP_DENSE_W4="1", MPCQP_BUILD="exp", PYTHONPATH=os.path.join(ROOT, "python-mpc_amd"))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True)
    got = json.loads(out.stdout.strip().splitlines()[-1])
    assert got["nb"] == 4 and got["bsize"] == [26, 25, 25, 28], got
    assert max(got["bsize"][0], got["bsize"][1]) <= 26 and max(got["bsize"][2], got["bsize"][3]) <= 28
    assert got["span"] <= 1 and got["amax"] == 5 and got["variant"] == 17, got
    env["MPCQP_BUILD"] = ""
    env.pop("MPCQP_DENSE_W4")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True)
    prod = json.loads(out.stdout.strip().splitlines()[-1])
    assert prod["bsize"] == [26, 25, 25, 28] and prod["span"] <= 1 and prod["amax"] == 5, prod
    env["MPCQP_BALANCE"] = "0"
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True)
    greedy = json.loads(out.stdout.strip().splitlines()[-1])
    assert greedy["bsize"] == [31, 30, 30, 13], greedy


def test_cfg2_workspace_carries_no_dense_inverse_rows():
    """The production library carves no dense-inverse rows (KParams::Kd, 256 x 54 doubles per
    instance) for cfg 2's four-block plan: that form is compiled into the experimental build
    only.  About 121 kB per instance (231 kB with the rows' 110,592 B), with and
    without MPCQP_DENSE_W4=1 (read once per process: children)."""
    code = r"""
import json
import osqp_amd
from osqp_amd import mpc
b = mpc.make_batch(2, B=2, seed=3)
P, _ = osqp_amd._drop_common_zeros(b["P"], b["Px"])
A, _ = osqp_amd._drop_common_zeros(b["A"], b["Ax"])
print(json.dumps(osqp_amd.plan_preview(P, A, **b["settings"])["bytes_per_instance"]))
"""
    for dk in ("0", "1"):
        env = dict(os.environ, MPCQP_DENSE_W4=dk, MPCQP_BUILD="", PYTHONPATH=os.path.join(ROOT, "python-mpc_amd"))
        out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True)
        bpi = json.loads(out.stdout.strip().splitlines()[-1])
        assert 115_000 < bpi < 125_000, bpi


def test_plan_preview_reports_a_rejected_elimination():
    """An eliminated plan the four-wave kernel cannot take (the slack layout at N = 30: 6
    blocks) is rejected with the failed preconditions named, and the plain plan is used."""
    P, q, A, l, u = mpc.slack_qp(30, np.zeros(5))
    info = osqp_amd.plan_preview(P, A, warm_start=True)
    assert info["plan_choice"] == 2 and info["n_eliminated"] == 0
    assert "nb = 6 (needs 4)" in info["note"] and "rejected" in info["note"]


def test_elimination_schur_complement_solves_the_full_system():
    """The algebra the four-wave kernel runs for an eliminated column j with parent p
    (factorize_w4, solve_w4_body): K_pp -= K_pj^2 / K_jj, b_p -= (K_pj / K_jj) b_j, then
    x_j = (b_j - K_pj x_p) / K_jj -- the exact solution of the full system K x = b."""
    b = mpc.make_batch(3, B=1, seed=5)
    P = b["P"]; A = b["A"]
    n = P.shape[0]
    Pf = (P + P.T - sparse.diags(P.diagonal())).toarray()
    rho = np.where(b["u"][0] - b["l"][0] < 1e-4, 100.0, 0.1)
    K = Pf + 1e-6 * np.eye(n) + A.T.toarray() @ np.diag(rho) @ A.toarray()
    rhs = np.random.default_rng(0).normal(size=n)
    x_ref = np.linalg.solve(K, rhs)
    Pz, _ = osqp_amd._drop_common_zeros(b["P"], b["Px"])
    Az, _ = osqp_amd._drop_common_zeros(b["A"], b["Ax"])
    nb, blk, var_pad, bsize, ne = osqp_amd.analyze(Pz, Az, eliminate=True)
    elim = np.flatnonzero(var_pad >= nb * blk)
    keep = np.flatnonzero(var_pad < nb * blk)
    Kr = K[np.ix_(keep, keep)].copy()
    br = rhs[keep].copy()
    pos = {v: i for i, v in enumerate(keep)}
    coup = {}
    for j in elim:
        nbrs = [p for p in np.flatnonzero(K[j]) if p != j]
        assert len(nbrs) <= 1
        if nbrs:
            p = nbrs[0]
            ec = K[p, j] / K[j, j]
            Kr[pos[p], pos[p]] -= K[p, j] * ec
            br[pos[p]] -= ec * rhs[j]
            coup[j] = (p, ec)
    xr = np.linalg.solve(Kr, br)
    x = np.empty(n)
    x[keep] = xr
    for j in elim:
        p, ec = coup.get(j, (None, 0.0))
        x[j] = rhs[j] / K[j, j] - (ec * x[p] if p is not None else 0.0)
    assert np.allclose(x, x_ref, rtol=1e-9, atol=1e-12)


def test_null_handle_is_einval():
    """Every handle entry point refuses a NULL handle with MPCQP_EINVAL (no device needed),
    the matrix-update and update-settings entries included."""
    import ctypes as C
    L = osqp_amd.lib()
    s = osqp_amd._make_settings()
    null = C.c_void_p()
    calls = [
        lambda: L.mpcqp_update_batch(null, None, None, None),
        lambda: L.mpcqp_update_matrices_batch(null, None, None, 0, None, None, 0),
        lambda: L.mpcqp_update_settings(null, C.byref(s), 0),
        lambda: L.mpcqp_warm_start_batch(null, None, None),
        lambda: L.mpcqp_solve_batch(null, None, None, None, None),
        lambda: L.mpcqp_get_info_batch(null, None, None, None, None, None),
        lambda: L.mpcqp_get_certificates(null, None, None),
        lambda: L.mpcqp_synchronize(null),
        lambda: L.mpcqp_set_one_shot(null, 1),
    ]
    for c in calls:
        assert c() == 1  # MPCQP_EINVAL (include/mpcqp.h)
    assert L.mpcqp_one_shot_applies(null) == 0
    with pytest.raises(ValueError, match="not initialized"):
        osqp_amd.OSQP().update_settings(eps_abs=1e-4)
    with pytest.raises(ValueError, match="not initialized"):
        osqp_amd.OSQPBatch().update(Px=np.ones((1, 3)))


def test_matrix_update_index_mapping_on_host():
    """OSQPBatch.update(Px=, Px_idx=) maps osqp's value indices (triu(P) CSC, explicit zeros
    included) to the device pattern, which drops entries zero in every instance: kept
    entries keep their order, a dropped one may only be set to zero (host logic, no device)."""
    b = osqp_amd.OSQPBatch()
    b.B = 2
    Px = np.array([[4.0, 0.0, 2.0, 1.0], [5.0, 0.0, 3.0, 0.0]])  # entry 1 zero in both instances
    kmap = osqp_amd._kept_index(Px)
    assert kmap.tolist() == [0, -1, 1, 2]
    vals, idx = b._matrix_values(np.array([[7.0, 0.0], [8.0, 0.0]]), np.array([3, 1]), kmap, 4, "P")
    assert idx.tolist() == [2] and vals.tolist() == [[7.0], [8.0]]
    vals, idx = b._matrix_values(np.arange(8.0).reshape(2, 4) * np.array([1, 0, 1, 1]), None, kmap, 4, "P")
    assert idx.tolist() == [0, 1, 2] and vals.shape == (2, 3)
    with pytest.raises(ValueError, match="zero in every instance"):
        b._matrix_values(np.array([[1.0], [0.0]]), np.array([1]), kmap, 4, "P")
    with pytest.raises(ValueError, match="greater than"):
        b._matrix_values(np.ones((2, 5)), np.arange(5), kmap, 4, "P")
    with pytest.raises(ValueError, match="out of range"):
        b._matrix_values(np.ones((2, 1)), np.array([4]), kmap, 4, "P")


def test_rotated_tile_row_network_round_trips():
    """ld_row16 / st_row16 (csrc/solve_phases.h): lane i reads column pair s ^ (i & 7) at step
    s and a three-stage conditional swap (bits 1, 2, 4 of i & 7) restores column order; the
    store applies the same involution before writing pair s ^ (i & 7).  The index model here
    checks that every row lands in column order and that a 16-lane group's reads of one step
    fall on distinct column pairs for distinct i & 7 (the 2-way bound of tools/lds_banks.py)."""
    def network(q, m):
        q = list(q)
        for bit in (1, 2, 4):
            if m & bit:
                for s in range(8):
                    if not s & bit:
                        q[s], q[s | bit] = q[s | bit], q[s]
        return q

    for i in range(32):
        m = i & 7
        row = [(i, 2 * c) for c in range(8)]            # pair c of row i
        loaded = [row[s ^ m] for s in range(8)]          # step s reads pair s ^ m
        assert network(loaded, m) == row
        out = [None] * 8
        for s, v in enumerate(network(row, m)):          # st_row16: q_s = pair s ^ m
            out[s ^ m] = v
        assert out == row
    for s in range(8):
        assert len({s ^ (i & 7) for i in range(8)}) == 8


def test_canonical_data_matches_scipy():
    """osqp_amd.canonical_data takes P's upper triangle from the CSC arrays directly and
    _drop_common_zeros drops the all-zero entries the same way: the same pattern, values and
    order as scipy.sparse.triu / eliminate_zeros (osqp-python's prepare_data), on random
    symmetric patterns with unsorted indices and explicit zeros."""
    from scipy import sparse
    rng = np.random.default_rng(0)
    for t in range(40):
        n, m = int(rng.integers(1, 40)), int(rng.integers(1, 40))
        M = sparse.random(n, n, density=0.3, random_state=int(rng.integers(1 << 30)), format="coo")
        M = (M + M.T).tocsc()
        if t % 3 == 0:
            M = sparse.csc_matrix((M.data[::-1].copy(), M.indices, M.indptr), shape=M.shape)
            M.has_sorted_indices = False
        A = sparse.random(m, n, density=0.2, random_state=int(rng.integers(1 << 30)), format="csc")
        P1, A1 = osqp_amd.canonical_data(M, A)
        P0 = sparse.triu(sparse.csc_matrix(M), format="csc")
        P0.sort_indices()
        assert np.array_equal(P1.indptr, P0.indptr) and np.array_equal(P1.indices, P0.indices)
        assert np.array_equal(P1.data, P0.data)
        V = rng.normal(size=(3, P1.nnz))
        V[:, ::4] = 0.0
        Mk, Vk = osqp_amd._drop_common_zeros(P1, V)
        keep = np.any(V != 0, axis=0)
        M0 = P1.copy()
        M0.data = keep.astype(float)
        M0.eliminate_zeros()
        M0.sort_indices()
        assert np.array_equal(Mk.indptr, M0.indptr) and np.array_equal(Mk.indices, M0.indices)
        assert np.array_equal(Vk, V[:, keep])
        assert np.array_equal(osqp_amd._kept_index(V)[keep], np.arange(int(keep.sum())))


def test_canonical_data_sums_duplicate_P_entries_like_triu():
    """canonical_data's fast upper triangle must match scipy.sparse.triu (what
    osqp-python's prepare_data takes), which sums duplicate entries; a P with a duplicated
    (0, 0) entry gave nnz 3 against triu's 2."""
    import scipy.sparse as sp
    from osqp_amd import canonical_data
    P = sp.csc_matrix((np.array([1.0, 2.0, 0.5, 3.0]), np.array([0, 0, 0, 1]), np.array([0, 2, 4])), shape=(2, 2))
    assert not P.has_canonical_format
    A = sp.csc_matrix(np.eye(2))
    Pc, _ = canonical_data(P, A)
    ref = sp.triu(P, format="csc")
    ref.sort_indices()
    assert Pc.nnz == ref.nnz == 3  # (0, 0) once, (0, 1), (1, 1)
    assert np.array_equal(Pc.indptr, ref.indptr) and np.array_equal(Pc.indices, ref.indices)
    assert np.array_equal(Pc.data, ref.data)
    assert Pc.toarray()[0, 0] == 3.0


def test_traffic_record_is_tied_to_the_measured_code(tmp_path, monkeypatch):
    """bench.py reports roofline.traffic only from a PMC record measured on the
    loaded library's code (code_sha16, tools/codeobj.py); another build's record is stale."""
    import json as _json
    import bench
    import osqp_amd
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import codeobj
    if not os.path.exists(osqp_amd.LIB_PATH):
        pytest.skip("libmpcqp.so not built")
    cur = codeobj.kernel_code_hash(osqp_amd.LIB_PATH, "mpcqp::k_setup_solve_w4")
    assert len(cur) == 16 and cur != codeobj.kernel_code_hash(osqp_amd.LIB_PATH, "mpcqp::k_solve_b")
    (tmp_path / "profiles").mkdir()
    rec = {"kernel": "mpcqp::k_setup_solve_w4", "bytes_per_launch": 123.0, "source": "test"}
    f = tmp_path / "profiles" / "traffic_w_b8.json"
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    for sha, stale in ((None, True), ("0123456789abcdef", True), (cur, False)):
        f.write_text(_json.dumps(dict(rec, code_sha16=sha)))
        t = bench.pmc_traffic("w", 8, "mpcqp::k_setup_solve_w4")
        assert bool(t.get("traffic_stale")) == stale, (sha, t)
        assert (t.get("bytes_per_launch") == 123.0) == (not stale)
    assert bench.pmc_traffic("w", 8, "mpcqp::k_solve_b") == {}  # a record of another kernel
