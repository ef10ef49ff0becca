# K1 bucket reduction A/B: weighted segments (default) vs TPST_K1_RED=2
# (two-level), parity at n = 20 / 24 fixtures, commit sweeps: tools/gpu_k1red.sh TAG
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-k1red}
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
PT="python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu"
TPST_K1_RED=2 timeout -k 10 600 $PT -k "commit or fullsize or batch or pedersen" > $OUT/gpu_tests_red2.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/commit_sweep.py 20 TPST_K1_RED=2 TPST_ACC_WAVES=4 TPST_ACC_WAVES=16 TPST_ACC_WAVES=4,TPST_K1_RED=2 > $OUT/sweep20.txt 2>&1 || exit 1
timeout -k 10 400 python -u tools/commit_sweep.py 24 TPST_K1_RED=2 > $OUT/sweep24.txt 2>&1 || exit 1
