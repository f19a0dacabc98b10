cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS -d gpurun_out/pmc_sq1 -o sq1 --output-format csv -- python3 tools/iter_cost.py --config 2 --batch 256 --iters 50 250 --reps 2 > gpurun_out/pmc_sq1.log 2>&1
