#!/bin/bash
# the launch-gap micro-benchmark under a kernel trace; prints the gaps per configuration
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/lgap; mkdir -p $out
timeout -k 10 60 tools/micro/launch_gap > $out/plain.txt 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace -d $out/kt -o kt --output-format csv -- tools/micro/launch_gap > $out/kt.log 2>&1 || exit 1
python3 - $out <<'PY'
import csv, glob, sys
out = sys.argv[1]
print(open(f'{out}/plain.txt').read())
f = glob.glob(f'{out}/kt/**/*kernel_trace.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
rows = [r for r in rows if 'launch_gap' in r['Kernel_Name'] or r['Kernel_Name'].startswith('void k<')]
names = ['plain 0', 'plain 8', 'plain 48', 'nt 0', 'nt 8', 'nt 48']
for c in range(6):
    grp = rows[c * 12:(c + 1) * 12]
    gaps = [(int(b['Start_Timestamp']) - int(a['End_Timestamp'])) / 1000 for a, b in zip(grp, grp[1:])]
    durs = [(int(a['End_Timestamp']) - int(a['Start_Timestamp'])) / 1000 for a in grp]
    print(names[c], 'gap us', [round(g, 1) for g in gaps], 'dur us', round(sum(durs) / len(durs), 1))
PY
