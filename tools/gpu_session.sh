#!/bin/bash
# One GPU session step list (through gpurun, from the repo root): the GPU test suite, the
# default bench line, and optional extra bench lines given as "name|args" words.  Every GPU
# step has its own time limit; the first failing step ends the script.
# usage: bash tools/gpu_session.sh <tag> <run_tests:0|1|k-expr> ["name|bench args" ...]
set -o pipefail
tag=$1; tests=$2; shift 2
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$tag
mkdir -p $out
if [ "$tests" = 1 ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
  tail -3 $out/pytest.log
elif [ "$tests" != 0 ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$tests" > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
  tail -3 $out/pytest.log
fi
for spec in "$@"; do
  name=${spec%%|*}; args=${spec#*|}
  [ "$args" = "$spec" ] && args=""
  eval "timeout -k 10 300 $args" > $out/$name.json 2> $out/$name.err || { echo "$name failed ($?)"; tail -20 $out/$name.err; exit 1; }
  tail -c 600 $out/$name.json; echo
done
echo done > $out/ok
