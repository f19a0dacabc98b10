# Same-box A/B of the long-horizon kernel: this build against ab/prev (another build's package):
# bit-identity of a cfg-5 batch (cold + warm), the cfg-5 bench (alternating), the one-QP latency
# leg and the B = 1 phase stamps.  usage: bash tools/ab_cfg5.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/$1; mkdir -p $o
PREV=$GRAFT_REPO_ROOT/ab/prev/python-mpc_amd
timeout -k 10 120 python3 tools/lchain_check.py $o/new.npz > $o/check.log 2>&1 || exit 1
MPCQP_PKG=$PREV timeout -k 10 120 python3 tools/lchain_check.py $o/prev.npz >> $o/check.log 2>&1 || exit 1
python3 tools/lchain_check.py --compare $o/new.npz $o/prev.npz >> $o/check.log 2>&1; rm -f $o/new.npz $o/prev.npz
for r in 1 2 3; do
  timeout -k 10 150 python3 bench.py --config 5 --no-cpu --no-pcie --no-latency --no-dispatch-ab --steps 5 --warmup 1 > $o/c5_new.$r.json 2>>$o/bench.err || exit 1
  MPCQP_PKG=$PREV timeout -k 10 150 python3 bench.py --config 5 --no-cpu --no-pcie --no-latency --no-dispatch-ab --steps 5 --warmup 1 > $o/c5_prev.$r.json 2>>$o/bench.err || exit 1
done
timeout -k 10 200 python3 tools/latency_ab.py 5 > $o/lat_new.json 2>>$o/bench.err || exit 1
timeout -k 10 120 python3 tools/phase_prof.py --config 5 --batch 1 > $o/phase_c5_b1.txt 2>&1 || exit 1
echo ok > $o/ok
