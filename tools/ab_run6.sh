# GPU tests + the commit with row blocks vs one block (TPST_COMMIT_BLOCKS=1), then the bench
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r6i}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $OUT/gpu_tests.log 2>&1 || exit 1
for i in 1 2; do
timeout -k 10 400 python -u tools/commit_sweep.py 24 TPST_COMMIT_BLOCKS=1 >> $OUT/ab_blocks24.txt 2>&1 || exit 1
timeout -k 10 400 python -u tools/commit_sweep.py 20 TPST_COMMIT_BLOCKS=1 >> $OUT/ab_blocks20.txt 2>&1 || exit 1
done
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
