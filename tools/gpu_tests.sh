# GPU parity tests only: tools/gpu_tests.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-run}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
if [ -n "$2" ]; then K="-k $2"; else K=""; fi
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu $K > $OUT/gpu_tests.log 2>&1
