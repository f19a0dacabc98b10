# Same-box A/B of the four-wave kernels (cfg 2 / 3): this build against ab/prev: bit-identity
# (cfg 2 and 3: cold, warm, one-shot) and alternating bench runs.  usage: bash tools/ab_w4.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/$1; mkdir -p $o
PREV=$GRAFT_REPO_ROOT/ab/prev/python-mpc_amd
for c in 2 3; do
  timeout -k 10 120 python3 tools/lchain_check.py $o/new$c.npz 512 $c >> $o/check.log 2>&1 || exit 1
  MPCQP_PKG=$PREV timeout -k 10 120 python3 tools/lchain_check.py $o/prev$c.npz 512 $c >> $o/check.log 2>&1 || exit 1
  python3 tools/lchain_check.py --compare $o/new$c.npz $o/prev$c.npz >> $o/check.log 2>&1; rm -f $o/new$c.npz $o/prev$c.npz
done
B="--no-cpu --no-pcie --no-latency"
for r in 1 2; do
  timeout -k 10 120 python3 bench.py $B --steps 30 --warmup 3 > $o/c2_new.$r.json 2>>$o/bench.err || exit 1
  MPCQP_PKG=$PREV timeout -k 10 120 python3 bench.py $B --steps 30 --warmup 3 > $o/c2_prev.$r.json 2>>$o/bench.err || exit 1
  timeout -k 10 150 python3 bench.py $B --no-dispatch-ab --config 3 --batch 65536 --steps 5 --warmup 1 > $o/c3_new.$r.json 2>>$o/bench.err || exit 1
  MPCQP_PKG=$PREV timeout -k 10 150 python3 bench.py $B --no-dispatch-ab --config 3 --batch 65536 --steps 5 --warmup 1 > $o/c3_prev.$r.json 2>>$o/bench.err || exit 1
  timeout -k 10 150 python3 bench.py $B --no-dispatch-ab --config 3 --batch 65536 --steps 5 --warmup 1 --no-one-shot > $o/c3p_new.$r.json 2>>$o/bench.err || exit 1
  MPCQP_PKG=$PREV timeout -k 10 150 python3 bench.py $B --no-dispatch-ab --config 3 --batch 65536 --steps 5 --warmup 1 --no-one-shot > $o/c3p_prev.$r.json 2>>$o/bench.err || exit 1
done
echo ok > $o/ok
