# confirmation on the committed tree: full GPU tests + smoke + bench (no CPU leg)
set -o pipefail
OUT=gpurun_out/${1:-confirm}
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no-cpu --steps 10 > $OUT/bench.json 2> $OUT/bench.err
