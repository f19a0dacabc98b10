#!/bin/bash
# Host-only sanitizer run of the planner (no GPU): dumps the sparsity patterns of the
# benchmark layouts and a few generic ones, builds plan.cpp with the driver under
# -fsanitize=address,undefined and plans each pattern with and without elimination.
set -e
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
T=$(mktemp -d)
trap 'rm -rf "$T"' EXIT
python3 - "$T" <<'PY'
import sys, os
sys.path.insert(0, os.path.join(os.environ.get("ROOT", "."), "python-mpc_amd"))
import numpy as np
from scipy import sparse
from osqp_amd import mpc, canonical_data
out = sys.argv[1]
def dump(name, P, A):
    P, A = canonical_data(P, A)
    with open(os.path.join(out, name + ".csc"), "wb") as f:
        np.array([P.shape[0], A.shape[0], P.nnz, A.nnz], np.int32).tofile(f)
        for a in (P.indptr, P.indices, A.indptr, A.indices):
            np.asarray(a, np.int32).tofile(f)
for cfg in (2, 3, 5):
    b = mpc.make_batch(cfg, B=2, seed=1)
    dump(f"cfg{cfg}", b["P"], b["A"])
rng = np.random.default_rng(7)
for k, (n, m, band) in enumerate([(40, 30, 2), (300, 200, 3), (1, 1, 0), (64, 0, 1)]):
    P = sparse.diags([np.ones(n)] + [np.full(n - d, 0.1) for d in range(1, band + 1)], [0] + list(range(1, band + 1)), (n, n))
    A = sparse.random(m, n, density=min(1.0, 3.0 / max(n, 1)), random_state=rng, format="csc") if m else sparse.csc_matrix((0, n))
    dump(f"generic{k}", P + P.T, A)
PY
g++ -O1 -g -std=c++17 -fsanitize=address,undefined -fno-omit-frame-pointer -I"$ROOT/python-mpc_amd/csrc" \
    "$ROOT/python-mpc_amd/csrc/plan.cpp" "$ROOT/tools/asan/plan_driver.cpp" -o "$T/plan_asan"
ASAN_OPTIONS=detect_leaks=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 "$T/plan_asan" "$T"/*.csc
