# round-4 closing session, part 1 on one box: full GPU tests, smoke, the
# default bench (with the CPU leg), the per-round open trace
#   bash tools/gpu_final4.sh TAG        (part 2: tools/gpu_prof_r4.sh TAG/prof)
set -o pipefail
TAG=${1:-final4}
OUT=gpurun_out/$TAG
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
TPST_OPEN_TRACE=1 timeout -k 10 120 python -u tools/prof_open.py 20 3 > $OUT/open_trace_stdout.txt 2> $OUT/open_trace.txt
