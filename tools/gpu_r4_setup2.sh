#!/bin/bash
# Round 4: setup latency after the one-wait setup path, the GPU suite, and the three-solver
# configs[0] records.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4_setup2}
mkdir -p $O
for c in 2 5; do
  timeout -k 10 120 python3 tools/setup_trace.py $c > $O/trace_cfg$c.txt 2>&1 || exit 1
  timeout -k 10 120 python3 tools/shim_latency.py --config $c --steps 120 > $O/shim_cfg$c.txt 2>&1 || exit 1
done
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 tools/diag_configs0_three.py --lo 1 --hi 1499 > $O/three_steps.txt 2>&1 || exit 1
timeout -k 10 300 python3 tools/diag_configs0_three.py --loops > $O/three_loops.txt 2>&1 || exit 1
tail -12 $O/trace_cfg5.txt; cat $O/shim_cfg*.txt $O/three_steps.txt $O/three_loops.txt
