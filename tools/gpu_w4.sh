#!/bin/bash
# four-wave kernel (variant 17) vs the default two-wave kernel (variant 10) on cfg 2:
# parity tests of the variant, then alternating benches on the same box
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$1; mkdir -p $out; reps=${2:-3}
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "alternative" > $out/pytest.log 2>&1 || exit $?
for i in $(seq 1 $reps); do
  timeout -k 10 200 python3 bench.py --no-cpu --no-dispatch-ab > $out/v10_$i.json 2> $out/v10_$i.err || exit $?
  MPCQP_VARIANT=17 timeout -k 10 200 python3 bench.py --no-cpu --no-dispatch-ab > $out/v17_$i.json 2> $out/v17_$i.err || exit $?
done
python3 - $out $reps <<'PY'
import json, sys
out, reps = sys.argv[1], int(sys.argv[2])
for k in ("v10", "v17"):
    v = [json.loads(open(f"{out}/{k}_{i}.json").read().strip().splitlines()[-1]) for i in range(1, reps + 1)]
    print(k, "value", [round(x["value"]) for x in v], "kernel_ms", [round(x["roofline"]["kernel_ms"], 4) for x in v],
          "iters", v[0]["config"]["iters_mean"], v[0]["config"]["iters_max"])
PY
if [ "${3:-0}" = 1 ]; then
  MPCQP_VARIANT=17 MPCQP_PHASE_PROF=1 timeout -k 10 200 python3 tools/phase_prof.py --config 2 > $out/phase_v17.txt 2>&1 || exit $?
fi
echo ok > $out/ok
