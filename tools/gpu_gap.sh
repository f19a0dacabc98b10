#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/gap; mkdir -p $out
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --no-cpu --no-dispatch-ab > $out/ev_$i.json 2>/dev/null || exit 1
  timeout -k 10 200 python3 bench.py --no-cpu --no-dispatch-ab --no-kernel-timing > $out/noev_$i.json 2>/dev/null || exit 1
done
timeout -k 10 240 rocprofv3 --kernel-trace -d $out/kt -o kt --output-format csv -- python3 bench.py --no-cpu --no-dispatch-ab --no-kernel-timing --steps 10 --warmup 2 > $out/kt.log 2>&1 || exit 1
python3 - $out <<'PY'
import json, sys, glob, csv
out = sys.argv[1]
for k in ('ev', 'noev'):
    v = [json.loads(open(f).read().strip().splitlines()[-1]) for f in sorted(glob.glob(f'{out}/{k}_*.json'))]
    print(k, [round(x['ms_per_step'], 4) for x in v], [round(x['roofline']['kernel_ms'], 4) for x in v])
f = glob.glob(f'{out}/kt/**/*kernel_trace.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
prev = None
gaps = []
for r in rows:
    if 'mpcqp' in r['Kernel_Name']:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        if prev: gaps.append((s - prev) / 1000)
        prev = e
    else:
        prev = None
print('gaps us', gaps)
PY
