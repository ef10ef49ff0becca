# the GPU test suite on the current build, then an interleaved opening A/B of
# the h-preparation stream's priority (greatest = default, TPST_OPEN_C_LEAST=1)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r6q}
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for i in 1 2 3; do
for C in 0 1; do
TPST_OPEN_C_LEAST=$C timeout -k 10 300 python -u tools/prof_open.py 20 5 > $OUT/t20_c${C}_$i.txt 2>&1 || exit 1
TPST_OPEN_C_LEAST=$C timeout -k 10 300 python -u tools/prof_open.py 24 3 > $OUT/t24_c${C}_$i.txt 2>&1 || exit 1
done
done
