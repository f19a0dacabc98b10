#!/bin/bash
# Profile pass (through gpurun): default bench with CPU baseline + rocprof kernel stats +
# FETCH/WRITE PMC passes for cfg 2, phase profiles cfg 2/3/5, cfg 3/5 benches.
# usage: bash tools/gpu_profile_all.sh <tag>
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$tag; mkdir -p $out
bash tools/profile_run.sh $tag/cfg2 || exit $?
MPCQP_PHASE_PROF=1 timeout -k 10 200 python3 tools/phase_prof.py --config 2 > $out/phase_cfg2.txt 2>&1 || exit $?
MPCQP_PHASE_PROF=1 timeout -k 10 200 python3 tools/phase_prof.py --config 3 --batch 8192 > $out/phase_cfg3.txt 2>&1 || exit $?
MPCQP_PHASE_PROF=1 timeout -k 10 200 python3 tools/phase_prof.py --config 5 --batch 2048 > $out/phase_cfg5.txt 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --config 3 --batch 65536 --steps 3 --warmup 1 > $out/bench_cfg3.json 2> $out/bench_cfg3.err || exit $?
timeout -k 10 300 python3 bench.py --config 5 --batch 8192 --steps 5 --warmup 1 > $out/bench_cfg5.json 2> $out/bench_cfg5.err || exit $?
echo ok > $out/ok
