cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/lat1
MPCQP_SETUP_TRACE=1 timeout -k 10 120 python3 tools/call_profile.py 5 20 > gpurun_out/lat1/trace.txt 2>&1
