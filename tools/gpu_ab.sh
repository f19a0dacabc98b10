#!/bin/bash
# A/B pass on the GPU box (through gpurun, from the repo root): GPU tests, then the
# cfg-2 bench and the phase profile for each MPCQP_VARIANT given.
# usage: bash tools/gpu_ab.sh <tag> <run_tests:0|1> <variant>...
set -o pipefail
tag=$1; tests=$2; shift 2
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$tag
mkdir -p $out
if [ "$tests" = 1 ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
fi
for v in "$@"; do
  MPCQP_VARIANT=$v timeout -k 10 200 python3 bench.py --no-cpu > $out/bench_v$v.json 2> $out/bench_v$v.err || exit $?
  MPCQP_VARIANT=$v MPCQP_PHASE_PROF=1 timeout -k 10 200 python3 tools/phase_prof.py --config 2 > $out/phase_v$v.txt 2>&1 || exit $?
done
echo done > $out/ok
