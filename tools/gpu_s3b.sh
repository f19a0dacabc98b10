set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/s3head2; mkdir -p $out
MPCQP_PHASE_PROF=1 timeout -k 10 200 python3 tools/phase_prof.py --config 2 > $out/phase_cfg2.txt 2>&1 || exit $?
MPCQP_PHASE_PROF=1 timeout -k 10 200 python3 tools/phase_prof.py --config 3 --batch 8192 > $out/phase_cfg3.txt 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --config 3 --batch 65536 --steps 3 --warmup 1 --no-cpu > $out/bench_cfg3.json 2> $out/bench_cfg3.err || exit $?
timeout -k 10 300 python3 bench.py --config 5 --batch 8192 --steps 5 --warmup 1 --no-cpu > $out/bench_cfg5.json 2> $out/bench_cfg5.err || exit $?
echo ok > $out/ok
