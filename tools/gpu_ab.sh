#!/bin/bash
# Same-box A/B/n of several builds (through gpurun, from the repo root): the cfg-2 bench
# alternated over the packages under ab/<name> and this tree's (".") <reps> times each,
# optionally after the GPU tests of this tree.
# usage: bash tools/gpu_ab.sh <tag> <run_tests:0|1> "<name> <name> ..." <reps> [bench args...]
set -o pipefail
tag=$1; tests=$2; names=$3; reps=$4; shift 4
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$tag
mkdir -p $out
if [ "$tests" = 1 ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
fi
for i in $(seq 1 $reps); do
  for n in $names; do
    if [ "$n" = "." ]; then pkg=$PWD/python-mpc_amd; else pkg=$PWD/ab/$n; fi
    MPCQP_PKG=$pkg timeout -k 10 200 python3 bench.py --no-cpu --no-dispatch-ab "$@" > $out/${n//./cur}_$i.json 2> $out/${n//./cur}_$i.err || exit $?
  done
done
python3 - $out $reps "$names" <<'PY'
import json, sys
out, reps, names = sys.argv[1], int(sys.argv[2]), sys.argv[3].split()
for n in names:
    k = n.replace(".", "cur")
    v = [json.loads(open(f"{out}/{k}_{i}.json").read().strip().splitlines()[-1]) for i in range(1, reps + 1)]
    print(k, "value", [round(x["value"]) for x in v], "kernel_ms", [round(x["roofline"]["kernel_ms"], 4) for x in v])
PY
echo done > $out/ok
