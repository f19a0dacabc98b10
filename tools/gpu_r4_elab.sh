#!/bin/bash
# Round 4: the configs[0] loops with the EL phase-A accumulation as one chain, and the cfg-3
# bench A/B against ab/base.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4_elab}
mkdir -p $O
timeout -k 10 300 python3 tools/diag_configs0_three.py --loops > $O/three_loops.txt 2>&1 || exit 1
cat $O/three_loops.txt
bash tools/gpu_ab.sh ${1:-r4_elab}/ab 0 "base ." 3 --config 3 --batch 65536 --steps 3 --warmup 1 || exit 1
