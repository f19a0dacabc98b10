set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/r5ab2; mkdir -p $out
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --no-cpu --no-dispatch-ab --no-pcie --no-latency > $out/base_$i.json 2> $out/base_$i.err || exit 1
  MPCQP_BALANCE=1 timeout -k 10 200 python3 bench.py --no-cpu --no-dispatch-ab --no-pcie --no-latency > $out/bal_$i.json 2> $out/bal_$i.err || exit 1
done
MPCQP_BALANCE=1 MPCQP_PHASE_PROF=1 timeout -k 10 200 python3 tools/phase_prof.py --config 2 > $out/ph_bal.txt 2>&1 || exit 1
python3 - <<'PY'
import json
for k in ("base","bal"):
    v=[json.loads(open(f"gpurun_out/r5ab2/{k}_{i}.json").read().strip().splitlines()[-1]) for i in (1,2,3)]
    print(k, [round(x["value"]) for x in v], [round(x["roofline"]["kernel_ms"],4) for x in v], [x["config"].get("iter_match_gpu") for x in v])
PY
head -20 $out/ph_bal.txt
