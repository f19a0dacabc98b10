#!/bin/bash
# Eight-wave kernel (variant 18) on MI355X: its parity test, then cfg 3 bench A/B against the default
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    -k "alternative and 18" > gpurun_out/w8_test.log 2>&1 || { echo "test failed"; tail -30 gpurun_out/w8_test.log; exit 1; }
tail -3 gpurun_out/w8_test.log
timeout -k 10 240 python bench.py --config 3 --batch 65536 --steps 3 --warmup 1 > gpurun_out/w8_b_def.json 2> gpurun_out/w8_b_def.err || exit 1
cat gpurun_out/w8_b_def.json
MPCQP_VARIANT=18 timeout -k 10 240 python bench.py --config 3 --batch 65536 --steps 3 --warmup 1 > gpurun_out/w8_b_18.json 2> gpurun_out/w8_b_18.err || exit 1
cat gpurun_out/w8_b_18.json
