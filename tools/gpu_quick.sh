set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$1; mkdir -p $out
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
MPCQP_PHASE_PROF=1 timeout -k 10 200 python3 tools/phase_prof.py --config 2 > $out/phase_cfg2.txt 2>&1 || exit $?
MPCQP_PHASE_PROF=1 timeout -k 10 200 python3 tools/phase_prof.py --config 3 --batch 8192 > $out/phase_cfg3.txt 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --no-cpu > $out/bench_cfg2.json 2> $out/bench_cfg2.err || exit $?
echo ok > $out/ok
