# Round-6 final records at HEAD: GPU suite, smoke, the default bench line, and one measurement
# pass per workload (bench line + kernel trace + PMC + SQ: tools/gpu_profile.sh), the persisting
# kernels' too.  usage: bash tools/r6_final.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
t=$1; o=gpurun_out/$t; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 1
bash tools/gpu_profile.sh $t/cfg2 || exit 1
bash tools/gpu_profile.sh $t/cfg3 --config 3 --batch 65536 --steps 3 --warmup 1 || exit 1
bash tools/gpu_profile.sh $t/cfg5 --config 5 --batch 8192 --steps 5 --warmup 1 || exit 1
bash tools/gpu_profile.sh $t/cfg2p --no-one-shot --no-cpu --no-pcie --no-latency || exit 1
bash tools/gpu_profile.sh $t/cfg3p --config 3 --batch 65536 --steps 3 --warmup 1 --no-one-shot --no-cpu --no-pcie --no-latency || exit 1
echo done > $o/ok
