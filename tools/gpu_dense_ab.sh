#!/bin/bash
# Same-box A/B of the four-wave kernel's dense-inverse form (MPCQP_DENSE_W4=1, the default)
# against the three-phase form (MPCQP_DENSE_W4=0), optionally after the GPU tests.
# usage: bash tools/gpu_dense_ab.sh <tag> <run_tests:0|1|k-expr> <reps> [bench args...]
set -o pipefail
tag=$1; tests=$2; reps=$3; shift 3
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$tag
mkdir -p $out
if [ "$tests" = 1 ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
  tail -3 $out/pytest.log
elif [ "$tests" != 0 ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$tests" > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
  tail -3 $out/pytest.log
fi
for i in $(seq 1 $reps); do
  for d in 1 0; do
    MPCQP_DENSE_W4=$d timeout -k 10 200 python3 bench.py --no-cpu --no-dispatch-ab "$@" > $out/d${d}_$i.json 2> $out/d${d}_$i.err || { tail -20 $out/d${d}_$i.err; exit 1; }
  done
done
python3 - $out $reps <<'PY'
import json, sys
out, reps = sys.argv[1], int(sys.argv[2])
for d in (1, 0):
    v = [json.loads(open(f"{out}/d{d}_{i}.json").read().strip().splitlines()[-1]) for i in range(1, reps + 1)]
    print(f"dense={d}", "value", [round(x["value"]) for x in v], "kernel_ms", [round(x["roofline"]["kernel_ms"], 4) for x in v],
          "solved", [x.get("solved_frac") for x in v])
PY
