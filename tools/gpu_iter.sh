# Iteration run on the GPU box: gpu tests, bench (no CPU leg), open profile.
# Stops at the first failing step.   bash tools/gpu_iter.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-it}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
K=""
if [ -n "$2" ]; then K="-k $2"; fi
timeout -k 10 400 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu $K > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -u bench.py --no-cpu --no-sharded > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
bash tools/gpu_prof_open.sh 20 || exit 1
cat $GRAFT_REPO_ROOT/gpurun_out/prof_open_20/stdout.txt
