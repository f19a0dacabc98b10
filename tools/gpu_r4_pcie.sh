#!/bin/bash
# Round 4: kernel + memory-copy trace of the bench (its PCIe leg at the end), and the
# configs[0] free-running test.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4_pcie}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "configs0" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o pcie -- python3 bench.py --no-cpu --no-dispatch-ab --steps 20 > $O/bench.json 2> $O/bench.err || exit 1
find $O/trace -name "*.csv" | head
