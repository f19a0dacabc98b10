# Same-box A/B of the dispatch predictor (KParams::odecay): this build against ab/prev on cfg 5
# and cfg 3 (the k_order path).  usage: bash tools/ab_order.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/$1; mkdir -p $o
PREV=$GRAFT_REPO_ROOT/ab/prev/python-mpc_amd
C5="--config 5 --no-cpu --no-pcie --no-latency --no-dispatch-ab --steps 10 --warmup 3"
C3="--config 3 --batch 65536 --no-cpu --no-pcie --no-latency --no-dispatch-ab --steps 6 --warmup 3"
for r in 1 2; do
  timeout -k 10 200 python3 bench.py $C5 > $o/c5_new.$r.json 2>>$o/err || exit 1
  MPCQP_PKG=$PREV timeout -k 10 200 python3 bench.py $C5 > $o/c5_prev.$r.json 2>>$o/err || exit 1
done
timeout -k 10 200 python3 bench.py $C3 > $o/c3_new.json 2>>$o/err || exit 1
MPCQP_PKG=$PREV timeout -k 10 200 python3 bench.py $C3 > $o/c3_prev.json 2>>$o/err || exit 1
echo ok > $o/ok
