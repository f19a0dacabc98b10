#!/bin/bash
# cfg 3 (B = 65536) and cfg 5 (B = 8192, warm) bench lines with the CPU baseline, through
# gpurun from the repo root.  usage: bash tools/gpu_cfg35.sh <tag>
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python3 bench.py --config 3 --batch 65536 --steps 3 --warmup 1 > $out/bench_cfg3.json 2> $out/bench_cfg3.err || exit $?
timeout -k 10 300 python3 bench.py --config 5 --batch 8192 --steps 5 --warmup 1 > $out/bench_cfg5.json 2> $out/bench_cfg5.err || exit $?
echo ok > $out/ok
