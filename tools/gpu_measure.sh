#!/bin/bash
# Round measurement pass on the GPU box (through gpurun, from the repo root): profile passes
# (tools/gpu_profile.sh) of the three single-GPU workloads, the bench-protocol sensitivity
# (jitter 2 % / 20 %, independent batches), cfg 4 (configs[3]) on one GPU as the whole
# 262144-instance job and as one rank's 32768 shard, and the F1 (--assemble) lines.
# usage: bash tools/gpu_measure.sh <tag>
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$tag
mkdir -p $out
b() {  # b <name> <limit> <bench args...>
    local name=$1 lim=$2; shift 2
    timeout -k 10 "$lim" python3 bench.py "$@" > $out/$name.json 2> $out/$name.err || { echo "$name failed ($?)"; exit 1; }
}
bash tools/gpu_profile.sh $tag/cfg2 || exit 1
bash tools/gpu_profile.sh $tag/cfg3 --config 3 --batch 65536 --steps 3 --warmup 1 || exit 1
bash tools/gpu_profile.sh $tag/cfg5 --config 5 --batch 8192 --steps 5 --warmup 1 || exit 1
b cfg2_jitter20 120 --no-cpu --jitter 0.2
b cfg2_independent 120 --no-cpu --independent
b cfg3_independent 200 --no-cpu --config 3 --batch 65536 --steps 3 --warmup 1 --independent
b cfg2_assemble 120 --no-cpu --assemble
b cfg3_assemble 200 --no-cpu --config 3 --batch 65536 --steps 3 --warmup 1 --assemble
b cfg4_1gpu_full 400 --no-cpu --config 4 --steps 5 --warmup 1 --no-dispatch-ab
b cfg4_rank_shard 200 --no-cpu --config 4 --batch 32768 --steps 5 --warmup 1
echo done > $out/ok
