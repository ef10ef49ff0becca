# GPU tests + smoke + default bench (+ optional rocprof of the bench): tools/gpu_test_bench.sh TAG [prof]
set -o pipefail
TAG=${1:-run}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > $OUT/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err && \
if [ "$2" = "prof" ]; then cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu > $OUT/bench_prof.json 2> $OUT/prof.err; fi
