set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/$1; mkdir -p $o
PREV=$GRAFT_REPO_ROOT/ab/prev/python-mpc_amd
timeout -k 10 120 python3 tools/lchain_check.py $o/new.npz > $o/check.log 2>&1 || exit 1
MPCQP_PKG=$PREV timeout -k 10 120 python3 tools/lchain_check.py $o/prev.npz >> $o/check.log 2>&1 || exit 1
python3 tools/lchain_check.py --compare $o/new.npz $o/prev.npz >> $o/check.log 2>&1; rm -f $o/new.npz $o/prev.npz
C="--config 5 --no-cpu --no-pcie --no-latency --no-dispatch-ab --steps 8 --warmup 3"
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py $C > $o/new.$r.json 2>>$o/err || exit 1
  MPCQP_PKG=$PREV timeout -k 10 200 python3 bench.py $C > $o/prev.$r.json 2>>$o/err || exit 1
done
echo ok > $o/ok
