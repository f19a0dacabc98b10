#!/bin/bash
# Round 4: the N > 1 bench path on the one-GPU box (every rank on GPU 0,
# MPCQP_BENCH_SHARE_GPU=1), plus a cfg-2 reference line of this box.
set -o pipefail
O=gpurun_out/r4_n2
mkdir -p $O
export MPCQP_BENCH_SHARE_GPU=1
timeout -k 10 240 python -u bench.py --gpus 2 --no-cpu > $O/cfg2_gpus2.json 2> $O/cfg2_gpus2.err && \
timeout -k 10 300 python -u bench.py --gpus 2 --config 4 --batch 65536 --steps 5 --warmup 1 --no-cpu > $O/cfg4_gpus2.json 2> $O/cfg4_gpus2.err && \
unset MPCQP_BENCH_SHARE_GPU && \
timeout -k 10 240 python -u bench.py --no-cpu > $O/cfg2_gpus1.json 2> $O/cfg2_gpus1.err
rc=$?
tail -c 600 $O/*.json
exit $rc
