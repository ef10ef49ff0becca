# GPU iteration: all -m gpu tests, the bench without its CPU leg, and the
# rocprofv3 kernel trace of the MSM leg (tools/msm_timeline.py reads it)
#   bash tools/gpu_iter.sh TAG [bench args]
set -o pipefail
TAG=${1:-it}
shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 400 python -u bench.py --no-cpu "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_msm -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-pst --no-sharded --no-groth16 --no-r1cs --steps 5 --warmup 2 > $OUT/prof_msm.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/msm_timeline.py $(ls $OUT/prof_msm/*kernel_trace.csv | head -1) > $OUT/msm_timeline.txt 2>&1; head -30 $OUT/msm_timeline.txt
