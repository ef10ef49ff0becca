# quick GPU iteration: selected tests + bench without the CPU leg
#   bash tools/gpu_quick.sh TAG "pytest -k expr" [bench args]
set -o pipefail
TAG=${1:-q}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu -k "$2" > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
shift 2
timeout -k 10 400 python -u bench.py --no-cpu "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
