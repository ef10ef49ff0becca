# MSM A/B of tagged libraries, then the opening on CU-partitioned streams
# (TPST_OPEN_CUMASK = CUs of the critical stream A; 0 = shared) and an
# opening parity check under the partition
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r6m}
shift
mkdir -p $OUT
cd $R
if [ $# -gt 0 ]; then
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "msm" > $OUT/msm_tests.log 2>&1 || exit 1
timeout -k 10 900 python -u tools/ab_libs.py 3 "$@" > $OUT/ab_msm.jsonl 2> $OUT/ab_msm.err || exit 1
fi
for i in 1 2; do
for K in 0 64 32 128; do
TPST_OPEN_CUMASK=$K timeout -k 10 300 python -u tools/prof_open.py 20 5 > $OUT/t20_k${K}_$i.txt 2>&1 || exit 1
TPST_OPEN_CUMASK=$K timeout -k 10 300 python -u tools/prof_open.py 24 3 > $OUT/t24_k${K}_$i.txt 2>&1 || exit 1
done
done
TPST_OPEN_CUMASK=64 timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_fullsize.py -x -q --timeout 300 --timeout-method thread -k "sqrt_pst or fullsize_commit_open" > $OUT/open_tests_k64.log 2>&1 || exit 1
