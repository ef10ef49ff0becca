# 2^20 open kernel timeline + per-round trace: tools/gpu_tl.sh TAG
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-tl}
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
TPST_OPEN_TRACE=1 timeout -k 10 120 python -u tools/prof_open.py 20 3 > $OUT/trace_stdout.txt 2> $OUT/trace.txt || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_open20 -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_open.py 20 3 > $OUT/prof_open20.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/open_timeline.py $OUT/prof_open20/run_kernel_trace.csv 600 > $OUT/open20_timeline.txt 2>&1
