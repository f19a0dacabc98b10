set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r1c
timeout -k 10 300 python3 bench.py --config 3 --batch 65536 --steps 3 --warmup 1 --no-cpu > gpurun_out/r1c/cfg3_65536.json 2> gpurun_out/r1c/cfg3.err || exit $?
timeout -k 10 300 python3 bench.py --config 5 --batch 8192 --steps 5 --warmup 1 --no-cpu > gpurun_out/r1c/cfg5_8192.json 2> gpurun_out/r1c/cfg5.err || exit $?
MPCQP_PHASE_PROF=1 timeout -k 10 200 python3 tools/phase_prof.py --config 3 --batch 8192 > gpurun_out/r1c/phase3.txt 2>&1 || exit $?
echo ok > gpurun_out/r1c/ok
