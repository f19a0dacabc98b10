# LDS factorisation chain: bit-identity (new on / new off / old build) and same-box timing
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r6o; mkdir -p $o
OLD=$GRAFT_REPO_ROOT/ab/old/python-mpc_amd
timeout -k 10 120 python3 tools/lchain_check.py $o/new.npz > $o/check.log 2>&1 || exit 1
MPCQP_LDS_CHAIN=0 timeout -k 10 120 python3 tools/lchain_check.py $o/off.npz >> $o/check.log 2>&1 || exit 1
MPCQP_PKG=$OLD timeout -k 10 120 python3 tools/lchain_check.py $o/old.npz >> $o/check.log 2>&1 || exit 1
python3 tools/lchain_check.py --compare $o/new.npz $o/off.npz >> $o/check.log 2>&1
python3 tools/lchain_check.py --compare $o/new.npz $o/old.npz >> $o/check.log 2>&1
for r in 1 2; do
  timeout -k 10 150 python3 bench.py --config 5 --no-cpu --no-pcie --no-latency --no-dispatch-ab --steps 5 --warmup 1 > $o/c5_new.$r.json 2>>$o/bench.err || exit 1
  MPCQP_PKG=$OLD timeout -k 10 150 python3 bench.py --config 5 --no-cpu --no-pcie --no-latency --no-dispatch-ab --steps 5 --warmup 1 > $o/c5_old.$r.json 2>>$o/bench.err || exit 1
  MPCQP_LDS_CHAIN=0 timeout -k 10 150 python3 bench.py --config 5 --no-cpu --no-pcie --no-latency --no-dispatch-ab --steps 5 --warmup 1 > $o/c5_off.$r.json 2>>$o/bench.err || exit 1
done
timeout -k 10 200 python3 tools/latency_ab.py 5 > $o/lat_new.json 2>>$o/bench.err || exit 1
MPCQP_LDS_CHAIN=0 timeout -k 10 200 python3 tools/latency_ab.py 5 > $o/lat_off.json 2>>$o/bench.err || exit 1
timeout -k 10 120 python3 tools/phase_prof.py --config 5 --batch 1 > $o/phase_c5_b1.txt 2>&1 || exit 1
echo ok > $o/ok
