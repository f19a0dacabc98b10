#!/bin/bash
# Round 4: the persistent fused kernel -- its tests, the GPU suite, and a same-box A/B of the
# cfg-2 bench: ab/base (before), this tree, this tree with MPCQP_PERSIST=0.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4_persist}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "persistent or fused" > $O/pytest_persist.log 2>&1 || { tail -30 $O/pytest_persist.log; exit 1; }
tail -1 $O/pytest_persist.log
b() {  # b <tag> <env> <pkg>
  env $2 MPCQP_PKG=$3 timeout -k 10 200 python3 bench.py --no-cpu --no-dispatch-ab --no-pcie > $O/$1.json 2> $O/$1.err || { echo "$1 failed"; tail -5 $O/$1.err; exit 1; }
}
for i in 1 2 3; do
  b base_$i MPCQP_PERSIST=1 $PWD/ab/base
  b cur_$i MPCQP_PERSIST=1 $PWD/python-mpc_amd
  b nop_$i MPCQP_PERSIST=0 $PWD/python-mpc_amd
done
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
for t in ("base", "cur", "nop"):
    v = [json.loads(open(f"{o}/{t}_{i}.json").read().strip().splitlines()[-1]) for i in (1, 2, 3)]
    print(t, [round(x["value"]) for x in v], [round(x["roofline"]["kernel_ms"], 4) for x in v])
PY
#timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
#tail -1 $O/pytest.log
