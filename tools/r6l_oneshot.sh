set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6l
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_one_shot.py tests/test_isa_shape.py > gpurun_out/r6l/pytest.log 2>&1 || exit 1
for r in 1 2; do
  for f in "" "--one-shot"; do
    timeout -k 10 120 python3 bench.py --no-cpu --no-pcie --no-latency --steps 30 --warmup 3 $f > gpurun_out/r6l/c2$f.$r.json 2>>gpurun_out/r6l/bench.err || exit 1
    timeout -k 10 180 python3 bench.py --config 3 --batch 65536 --no-cpu --no-pcie --no-latency --no-dispatch-ab --steps 5 --warmup 1 $f > gpurun_out/r6l/c3$f.$r.json 2>>gpurun_out/r6l/bench.err || exit 1
  done
done
bash tools/gpu_profile.sh r6l/cfg2one --one-shot && bash tools/gpu_profile.sh r6l/cfg3one --config 3 --batch 65536 --steps 3 --warmup 1 --one-shot
