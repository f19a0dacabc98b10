#!/bin/bash
# One measurement pass on the GPU box (run through gpurun from the repo root):
#   bench line (with CPU baseline), rocprofv3 kernel-trace stats of the same command,
#   separate FETCH_SIZE / WRITE_SIZE PMC passes -> profiles/traffic_<workload>_b<B>.json
# usage: bash tools/profile_run.sh <tag> [bench args...]
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python3 bench.py "$@" > $out/bench.json 2> $out/bench.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/kt -o kt --output-format csv -- python3 bench.py --no-cpu --no-dispatch-ab --steps 10 --warmup 2 "$@" > $out/kt.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d $out/pmc_f -o f --output-format csv -- python3 bench.py --no-cpu --no-dispatch-ab --steps 2 --warmup 1 "$@" > $out/pmc_f.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d $out/pmc_w -o w --output-format csv -- python3 bench.py --no-cpu --no-dispatch-ab --steps 2 --warmup 1 "$@" > $out/pmc_w.log 2>&1 || exit $?
echo done > $out/ok
