# GPU test suite on the current build, then an interleaved commit + open A/B
# of the current library against a tagged baseline (TPST_LIB_PATH)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r6s}
BASE=${2:-testudo_amd/libtpst_old.so}
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for i in 1 2 3; do
TPST_LIB_PATH=$R/$BASE timeout -k 10 300 python -u tools/prof_open.py 20 5 > $OUT/t20_old_$i.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/prof_open.py 20 5 > $OUT/t20_new_$i.txt 2>&1 || exit 1
TPST_LIB_PATH=$R/$BASE timeout -k 10 300 python -u tools/prof_open.py 24 3 > $OUT/t24_old_$i.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/prof_open.py 24 3 > $OUT/t24_new_$i.txt 2>&1 || exit 1
done
