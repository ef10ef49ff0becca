# unsharded opening rebase (TPST_OPEN_REBASE = L): the opening parity tests
# with L = 8 (every size with C > 8 rebases), then an interleaved A/B of L
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r6ab}
mkdir -p $OUT
cd $R
TPST_OPEN_REBASE=8 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_rebase8.log 2>&1 || exit 1
for i in 1 2; do
for L in 0 64 256 16; do
TPST_OPEN_REBASE=$L timeout -k 10 300 python -u tools/prof_open.py 20 5 > $OUT/t20_L${L}_$i.txt 2>&1 || exit 1
TPST_OPEN_REBASE=$L timeout -k 10 300 python -u tools/prof_open.py 24 3 > $OUT/t24_L${L}_$i.txt 2>&1 || exit 1
done
done
