# kernel-time summary of the cfg 5 bench for this tree and for ab/prev (A/B of one kernel's change)
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/$1; mkdir -p $o
PREV=$GRAFT_REPO_ROOT/ab/prev/python-mpc_amd
C="--config 5 --no-cpu --no-pcie --no-latency --no-dispatch-ab --steps 4 --warmup 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/new -o run -- python3 bench.py $C > $o/new.json 2>>$o/err || exit 1
MPCQP_PKG=$PREV timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prev -o run -- python3 bench.py $C > $o/prev.json 2>>$o/err || exit 1
find $o -name '*kernel_trace.csv' -delete
echo ok > $o/ok
