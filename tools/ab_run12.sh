# placement of the PST proof of q in the opening (TPST_PSTQ_AT: 0 = stream B
# in round 0, 1 / 2 / 3 = stream C in round 0 / m - 2 / m / 2), interleaved,
# then the opening parity tests under each non-default placement
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r6r}
mkdir -p $OUT
cd $R
for i in 1 2; do
for Q in 0 1 2 3; do
TPST_PSTQ_AT=$Q timeout -k 10 300 python -u tools/prof_open.py 20 5 > $OUT/t20_q${Q}_$i.txt 2>&1 || exit 1
TPST_PSTQ_AT=$Q timeout -k 10 300 python -u tools/prof_open.py 24 3 > $OUT/t24_q${Q}_$i.txt 2>&1 || exit 1
done
done
for Q in 1 2 3; do
TPST_PSTQ_AT=$Q timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_fullsize.py tests/test_sharded_open.py -x -q --timeout 300 --timeout-method thread -k "sqrt_pst or fullsize_commit_open or 11-2 or 12-4 or 13-8" > $OUT/open_tests_q$Q.log 2>&1 || exit 1
done
