# one box, everything: microbenchmarks, full GPU tests, smoke, bench (no CPU
# leg), gather experiment, 2-rank shared-GPU rehearsal, then the profiles
#   bash tools/gpu_all4.sh TAG
set -o pipefail
TAG=${1:-all4}
OUT=gpurun_out/$TAG
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
timeout -k 10 120 python -u tools/mb_fq29.py > $OUT/mb_fq29.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || exit 1
TPST_GATHER_MASK=12 timeout -k 10 300 python -u bench.py --no-cpu --no-pst --no-r1cs --no-groth16 --steps 5 > $OUT/gmask12.json 2> $OUT/gmask12.err || exit 1
TPST_BENCH_SHARED_GPU=1 timeout -k 10 500 python -u bench.py --gpus 2 --no-cpu --steps 5 > $OUT/bench_shared2.json 2> $OUT/bench_shared2.err || exit 1
bash tools/gpu_prof_r4.sh $TAG/prof
