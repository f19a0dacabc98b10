#!/bin/bash
# Same-box A/B of environment switches (through gpurun, from the repo root): the bench with
# each "name|ENV=VAL ..." spec (empty env: the default) alternated `reps` times.
# usage: bash tools/ab_env.sh <tag> <reps> "<bench args>" "name|env" "name|env" ...
set -o pipefail
tag=$1; reps=$2; bargs=$3; shift 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$tag; mkdir -p $out
for i in $(seq 1 $reps); do
  for spec in "$@"; do
    name=${spec%%|*}; envs=${spec#*|}
    env $envs timeout -k 10 200 python3 bench.py --no-cpu --no-dispatch-ab --no-pcie --no-latency $bargs > $out/${name}_$i.json 2> $out/${name}_$i.err || { echo "$name failed"; tail -5 $out/${name}_$i.err; exit 1; }
  done
done
python3 - $out $reps "$@" <<'PY'
import json, sys
out, reps = sys.argv[1], int(sys.argv[2])
for spec in sys.argv[3:]:
    k = spec.split("|")[0]
    v = [json.loads(open(f"{out}/{k}_{i}.json").read().strip().splitlines()[-1]) for i in range(1, reps + 1)]
    print(k, "value", [round(x["value"]) for x in v], "kernel_ms", [round(x["roofline"]["kernel_ms"], 4) for x in v])
PY
