# setup time against batch size and Ruiz pass count, this tree (and ab/prev with "prev")
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/$1; mkdir -p $o
for sc in 0 1 10; do
  SCAN_SCALING=$sc timeout -k 10 200 python3 tools/setup_scan.py 5 1 256 512 1024 8192 >> $o/new.txt 2>&1 || exit 1
done
if [ "$2" = prev ]; then
  MPCQP_PKG=$GRAFT_REPO_ROOT/ab/prev/python-mpc_amd timeout -k 10 200 python3 tools/setup_scan.py 5 > $o/prev.txt 2>&1 || exit 1
fi
echo ok > $o/ok
