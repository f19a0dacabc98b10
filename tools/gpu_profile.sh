#!/bin/bash
# One measurement pass on the GPU box (run through gpurun, from the repo root):
#   the bench line (with its CPU baseline)                         -> bench.json
#   rocprofv3 --kernel-trace --stats of the same workload          -> kt/
#   --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate passes         -> pmc_f/, pmc_w/, traffic.json
#   two SQ passes: where the waves' cycles go, the LDS counters    -> sq1/, sq2/, sq.json
# Every GPU step has its own time limit; the first failing step ends the script.
# usage: bash tools/gpu_profile.sh <tag> [bench args...]
set -o pipefail
tag=$1; shift
args=("$@")
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$tag
mkdir -p $out
step() {  # step <name> <timeout> <cmd...>: stdout+stderr to $out/<name>.log
    local name=$1 lim=$2; shift 2
    timeout -k 10 "$lim" "$@" > "$out/$name.log" 2>&1
    local rc=$?
    if [ $rc -ne 0 ]; then echo "$name failed ($rc)" | tee -a "$out/failed"; exit $rc; fi
}
timeout -k 10 300 python3 bench.py "${args[@]}" > $out/bench.json 2> $out/bench.err || { echo "bench failed"; exit 1; }
short=(--no-cpu --no-dispatch-ab --no-pcie --steps 4 --warmup 1 "${args[@]}")
step kt 240 rocprofv3 --kernel-trace --stats -d $out/kt -o kt --output-format csv -- python3 bench.py --no-cpu --no-dispatch-ab --no-pcie --steps 10 --warmup 2 "${args[@]}"
step pmc_f 120 rocprofv3 --pmc FETCH_SIZE -d $out/pmc_f -o f --output-format csv -- python3 bench.py "${short[@]}"
step pmc_w 120 rocprofv3 --pmc WRITE_SIZE -d $out/pmc_w -o w --output-format csv -- python3 bench.py "${short[@]}"
step sq1 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS -d $out/sq1 -o sq1 --output-format csv -- python3 bench.py "${short[@]}"
step sq2 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE -d $out/sq2 -o sq2 --output-format csv -- python3 bench.py "${short[@]}"
python3 tools/pmc_summary.py $out > $out/summary.txt 2>&1
echo done > $out/ok
