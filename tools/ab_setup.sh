# A/B of a batch-setup change (cfg 5): bit-identity on a cold + warm batch, the setup time
# against the batch size, and the cfg-5 bench, alternating this tree and ab/prev
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/$1; mkdir -p $o
PREV=$GRAFT_REPO_ROOT/ab/prev/python-mpc_amd
timeout -k 10 120 python3 tools/lchain_check.py $o/new.npz 2048 > $o/check.log 2>&1 || exit 1
MPCQP_PKG=$PREV timeout -k 10 120 python3 tools/lchain_check.py $o/prev.npz 2048 >> $o/check.log 2>&1 || exit 1
python3 tools/lchain_check.py --compare $o/new.npz $o/prev.npz >> $o/check.log 2>&1; rm -f $o/new.npz $o/prev.npz
timeout -k 10 200 python3 tools/setup_scan.py 5 1 256 512 8192 > $o/scan_new.txt 2>&1 || exit 1
MPCQP_SETUP_FULL=1 timeout -k 10 200 python3 tools/setup_scan.py 5 1 256 512 8192 > $o/scan_full.txt 2>&1 || exit 1
MPCQP_PKG=$PREV timeout -k 10 200 python3 tools/setup_scan.py 5 1 256 512 8192 > $o/scan_prev.txt 2>&1 || exit 1
C="--config 5 --no-cpu --no-pcie --no-latency --no-dispatch-ab --steps 8 --warmup 3"
for r in 1 2; do
  timeout -k 10 200 python3 bench.py $C > $o/new.$r.json 2>>$o/err || exit 1
  MPCQP_PKG=$PREV timeout -k 10 200 python3 bench.py $C > $o/prev.$r.json 2>>$o/err || exit 1
done
echo ok > $o/ok
