#!/bin/bash
# step-gap A/B: the cfg-2 bench without kernel timing for ab/<names> (3 runs each), then a
# kernel trace of the last name's package with the gaps between its solve kernels
set -o pipefail
names=$1; shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/gapab; mkdir -p $out
bash tools/gpu_ab.sh gapab_runs 0 "$names" 3 --no-kernel-timing "$@" || exit 1
last=${names##* }
MPCQP_PKG=$PWD/ab/$last timeout -k 10 240 rocprofv3 --kernel-trace -d $out/kt -o kt --output-format csv -- python3 bench.py --no-cpu --no-dispatch-ab --no-kernel-timing --steps 10 --warmup 2 "$@" > $out/kt.log 2>&1 || exit 1
python3 - $out <<'PY'
import csv, glob, sys
out = sys.argv[1]
f = glob.glob(f'{out}/kt/**/*kernel_trace.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
prev, gaps = None, []
for r in rows:
    if 'mpcqp' in r['Kernel_Name']:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        if prev: gaps.append(round((s - prev) / 1000, 1))
        prev = e
    else:
        prev = None
print('gaps us', gaps)
PY
