# K1 reduction form at 2^20 (TPST_K1_RED_LANE), interleaved commit + open,
# plus a kernel trace of each setting
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r6z}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
for i in 1 2 3; do
for L in 0 1; do
TPST_K1_RED_LANE=$L timeout -k 10 300 python -u tools/prof_open.py 20 5 > $OUT/t20_lane${L}_$i.txt 2>&1 || exit 1
done
done
for L in 0 1; do
cd /tmp && TPST_K1_RED_LANE=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_lane$L -o run -- python3 $R/tools/prof_open.py 20 3 > $OUT/prof_lane$L.log 2>&1 || exit 1
done
cd $R && TPST_K1_RED_LANE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_fullsize.py -x -q --timeout 300 --timeout-method thread -k "sqrt_pst or fullsize_commit_open or batch" > $OUT/tests_lane1.log 2>&1 || exit 1
