# K1 level-1 reduction: quads at 16 (default) vs lanes at 8 (TPST_K1_RED_LG=3 TPST_K1_RED_LANE=1), 2^20 + 2^24
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r6ah}
mkdir -p $OUT
cd $R
for i in 1 2 3; do
timeout -k 10 300 python -u tools/prof_open.py 20 5 > $OUT/t20_base_$i.txt 2>&1 || exit 1
TPST_K1_RED_LG=3 TPST_K1_RED_LANE=1 timeout -k 10 300 python -u tools/prof_open.py 20 5 > $OUT/t20_lg3lane_$i.txt 2>&1 || exit 1
done
for i in 1 2; do
timeout -k 10 300 python -u tools/prof_open.py 24 3 > $OUT/t24_base_$i.txt 2>&1 || exit 1
TPST_K1_RED_LG=3 TPST_K1_RED_LANE=1 timeout -k 10 300 python -u tools/prof_open.py 24 3 > $OUT/t24_lg3lane_$i.txt 2>&1 || exit 1
done
TPST_K1_RED_LG=3 TPST_K1_RED_LANE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_fullsize.py tests/test_boundary.py -x -q --timeout 300 --timeout-method thread -k "sqrt_pst or fullsize_commit_open or batch" > $OUT/tests.log 2>&1 || exit 1
