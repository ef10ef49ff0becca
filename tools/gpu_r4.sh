# round-4 GPU session: tests, smoke, bench, shared-GPU 2-rank rehearsal, skew probe
# tools/gpu_r4.sh TAG
set -o pipefail
TAG=${1:-r4}
OUT=gpurun_out/$TAG
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
timeout -k 10 120 python -u tools/mb_fq29.py > $OUT/mb_fq29.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 200 python -u tools/msm_skew_probe.py > $OUT/skew.log 2>&1 && \
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err && \
TPST_BENCH_SHARED_GPU=1 timeout -k 10 400 python -u bench.py --gpus 2 --no-cpu --steps 5 > $OUT/bench_shared2.json 2> $OUT/bench_shared2.err
