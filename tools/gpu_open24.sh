# 2^24 open: per-round host trace + kernel timeline: bash tools/gpu_open24.sh TAG
set -o pipefail
TAG=${1:-open24}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
TPST_OPEN_TRACE=1 timeout -k 10 200 python -u tools/prof_open.py 24 3 > $OUT/open_trace_stdout.txt 2> $OUT/open_trace.txt || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_open24 -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_open.py 24 3 > $OUT/prof_open24.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/open_timeline.py $OUT/prof_open24/run_kernel_trace.csv 900 > $OUT/open24_timeline.txt 2>&1
