#!/bin/bash
# quick GPU pass: GPU tests, cfg-2 bench, cfg-2 phase profile (usage: bash tools/gpu_quick2.sh <tag> [tests:0|1])
set -o pipefail
tag=$1; tests=${2:-1}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$tag; mkdir -p $out
if [ "$tests" = 1 ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
fi
timeout -k 10 200 python3 bench.py --no-cpu > $out/bench_cfg2.json 2> $out/bench_cfg2.err || exit $?
MPCQP_PHASE_PROF=1 timeout -k 10 200 python3 tools/phase_prof.py --config 2 > $out/phase_cfg2.txt 2>&1 || exit $?

if [ "${3:-0}" = 1 ]; then
  MPCQP_PHASE_PROF=1 timeout -k 10 200 python3 tools/phase_prof.py --config 3 --batch 8192 > $out/phase_cfg3.txt 2>&1 || exit $?
  timeout -k 10 300 python3 bench.py --config 3 --batch 65536 --steps 3 --warmup 1 --no-cpu > $out/bench_cfg3.json 2> $out/bench_cfg3.err || exit $?
  timeout -k 10 300 python3 bench.py --config 5 --batch 8192 --steps 5 --warmup 1 --no-cpu > $out/bench_cfg5.json 2> $out/bench_cfg5.err || exit $?
fi
echo ok2 > $out/ok2
