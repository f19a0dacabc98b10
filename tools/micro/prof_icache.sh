# PMC passes on a solve workload (run through gpurun from the repo root):
# instruction-cache behaviour and where waves wait.  usage: bash tools/micro/prof_icache.sh <tag> <bench args...>
tag=$1; shift
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 200 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH -d $out/ic -o ic --output-format csv -- python3 bench.py --no-cpu --steps 2 --warmup 1 "$@" > $out/ic.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS -d $out/sq -o sq --output-format csv -- python3 bench.py --no-cpu --steps 2 --warmup 1 "$@" > $out/sq.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_INSTS_FLAT -d $out/sq2 -o sq2 --output-format csv -- python3 bench.py --no-cpu --steps 2 --warmup 1 "$@" > $out/sq2.log 2>&1 || exit $?
echo done > $out/ok
