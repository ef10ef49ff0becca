# tests + smoke + wave-engine stage microbench + bench on the GPU box
#   bash tools/gpu_quick2.sh TAG
set -o pipefail
TAG=${1:-q}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/mb_wave.py > $OUT/mb_wave.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/mb_lat.py > $OUT/mb_lat.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
