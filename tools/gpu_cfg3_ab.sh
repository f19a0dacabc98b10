#!/bin/bash
# cfg 3 kernel A/B: benches (B = 65536) and phase profiles (B = 8192) per variant
# usage: bash tools/gpu_cfg3_ab.sh <tag> "<variants>"
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$1; mkdir -p $out
for v in ${2:-2 14}; do
  MPCQP_VARIANT=$v timeout -k 10 300 python3 bench.py --config 3 --batch 65536 --steps 3 --warmup 1 --no-cpu --no-dispatch-ab > $out/bench_cfg3_v$v.json 2> $out/bench_cfg3_v$v.err || exit $?
  MPCQP_VARIANT=$v MPCQP_PHASE_PROF=1 timeout -k 10 200 python3 tools/phase_prof.py --config 3 --batch 8192 > $out/phase_cfg3_v$v.txt 2>&1 || exit $?
done
echo ok > $out/ok
