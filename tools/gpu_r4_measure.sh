#!/bin/bash
# Round 4 measurement pass: tools/gpu_profile.sh on the three single-GPU workloads.
set -o pipefail
tag=${1:-r4_m}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_profile.sh $tag/cfg2 || exit 1
bash tools/gpu_profile.sh $tag/cfg5 --config 5 --batch 8192 --steps 5 --warmup 1 || exit 1
bash tools/gpu_profile.sh $tag/cfg3 --config 3 --batch 65536 --steps 3 --warmup 1 || exit 1
for c in cfg2 cfg5 cfg3; do head -12 gpurun_out/$tag/$c/summary.txt; done
