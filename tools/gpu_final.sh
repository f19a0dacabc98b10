#!/bin/bash
# Round-end rehearsal on the GPU box (through gpurun, from the repo root): the driver's
# GPU tier in order -- pytest -m gpu, smoke(), the default bench -- plus the bench through
# torch.distributed.run with one rank (the launcher path of the scaling runs).
set -o pipefail
tag=${1:-final}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py > $out/bench.json 2> $out/bench.err || exit $?
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 10 --warmup 2 > $out/bench_dist1.json 2> $out/bench_dist1.err || exit $?
echo ok > $out/ok
