#!/bin/bash
# GPU tests + cfg 5 bench and phase profile (usage: bash tools/gpu_cfg5.sh <tag>)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$1; mkdir -p $out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --config 5 --batch 8192 --steps 5 --warmup 1 --no-cpu > $out/bench_cfg5.json 2> $out/bench_cfg5.err || exit $?
MPCQP_PHASE_PROF=1 timeout -k 10 200 python3 tools/phase_prof.py --config 5 --batch 2048 > $out/phase_cfg5.txt 2>&1 || exit $?
echo ok > $out/ok
