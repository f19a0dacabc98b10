#!/bin/bash
# cfg 3 (B = 65536) with each kernel variant that fits its plan (A/B only)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$1; mkdir -p $out
for v in ${2:-2 3 11 14}; do
  MPCQP_VARIANT=$v timeout -k 10 300 python3 bench.py --config 3 --batch 65536 --steps 3 --warmup 1 --no-cpu > $out/bench_cfg3_v$v.json 2> $out/bench_cfg3_v$v.err || exit $?
done
echo ok > $out/ok
