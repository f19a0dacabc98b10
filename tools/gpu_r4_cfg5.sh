#!/bin/bash
# Round 4: the split two-sided factorisation (solve_big.hip::factorize2s) -- the GPU suite, a
# same-box A/B of the cfg-5 bench against ab/base, and the cfg-5 single-QP setup trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4_cfg5}
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  for t in base cur; do
    if [ $t = base ]; then pkg=$PWD/ab/${AB_BASE:-base}; else pkg=$PWD/python-mpc_amd; fi
    MPCQP_PKG=$pkg timeout -k 10 300 python3 bench.py --no-cpu --no-dispatch-ab --config 5 --steps 5 --warmup 1 > $O/${t}_$i.json 2> $O/${t}_$i.err || { echo "$t failed"; tail -5 $O/${t}_$i.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], round(d['value']), round(d['roofline']['kernel_ms'],3), d['config']['iters_mean'])" $O/${t}_$i.json $t
  done
done
timeout -k 10 120 python3 tools/setup_trace.py 5 > $O/trace_cfg5.txt 2>&1 || exit 1
tail -9 $O/trace_cfg5.txt
