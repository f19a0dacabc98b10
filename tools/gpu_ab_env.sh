#!/bin/bash
# Same-box A/B of builds x environments: each argument "name:pkg:ENV=V,ENV=V" (pkg "." = this
# tree's package, else ab/<pkg>), the cfg-2-style bench alternated <reps> times.
# usage: bash tools/gpu_ab_env.sh <tag> <reps> "<bench args>" spec spec ...
set -o pipefail
tag=$1; reps=$2; bargs=$3; shift 3
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$tag
mkdir -p $out
for i in $(seq 1 $reps); do
  for spec in "$@"; do
    IFS=: read -r name pkg envs <<< "$spec"
    if [ "$pkg" = "." ]; then pp=$PWD/python-mpc_amd; else pp=$PWD/ab/$pkg; fi
    env $(echo "$envs" | tr ',' ' ') MPCQP_PKG=$pp timeout -k 10 200 python3 bench.py --no-cpu --no-dispatch-ab $bargs > $out/${name}_$i.json 2> $out/${name}_$i.err || { tail -20 $out/${name}_$i.err; exit 1; }
  done
done
python3 - $out $reps "$@" <<'PY'
import json, sys
out, reps, specs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
for sp in specs:
    k = sp.split(":")[0]
    v = [json.loads(open(f"{out}/{k}_{i}.json").read().strip().splitlines()[-1]) for i in range(1, reps + 1)]
    print(k, "value", [round(x["value"]) for x in v], "kernel_ms", [round(x["roofline"]["kernel_ms"], 4) for x in v],
          "solved", [x.get("solved_frac") for x in v])
PY
