# PMC counters of the batch setup kernel (cfg 5, B = 8192), one pass per counter group
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/$1; mkdir -p $o
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES --output-format csv -d $o/p1 -o run -- python3 tools/setup_scan.py 5 8192 > $o/p1.txt 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $o/p2 -o run -- python3 tools/setup_scan.py 5 8192 > $o/p2.txt 2>&1 || exit 1
echo ok > $o/ok
