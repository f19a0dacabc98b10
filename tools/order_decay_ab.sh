set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r6zg; mkdir -p $o
for r in 1 2; do for d in 0 4 6 7; do
  MPCQP_ORDER_DECAY=$d timeout -k 10 200 python3 bench.py --config 5 --no-cpu --no-pcie --no-latency --no-dispatch-ab --steps 8 --warmup 3 > $o/c5_d$d.$r.json 2>>$o/err || exit 1
done; done
for d in 0 6; do MPCQP_ORDER_DECAY=$d timeout -k 10 200 python3 bench.py --config 3 --batch 65536 --no-cpu --no-pcie --no-latency --no-dispatch-ab --steps 6 --warmup 3 > $o/c3_d$d.json 2>>$o/err || exit 1; done
echo ok > $o/ok
