#!/bin/bash
# Round 4: the GPU suite at HEAD, then the fresh-object-per-call latency (plan cache + pool)
# for cfg 2 / 3 / 5.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4_setup}
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for c in 2 3 5; do
  timeout -k 10 120 python3 tools/setup_latency_probe.py $c > $O/probe_cfg$c.txt 2>&1 || exit 1
  timeout -k 10 120 python3 tools/shim_latency.py --config $c --steps 120 > $O/shim_cfg$c.txt 2>&1 || exit 1
done
cat $O/probe_cfg*.txt $O/shim_cfg*.txt
