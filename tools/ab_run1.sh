set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6c
mkdir -p $OUT
cd $R
TPST_LIB_PATH=$R/testudo_amd/libtpst_m3.so timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "msm" > $OUT/m3_msm_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/ab_libs.py 3 main=testudo_amd/libtpst.so m3=testudo_amd/libtpst_m3.so > $OUT/ab_msm.jsonl 2> $OUT/ab_msm.err || exit 1
timeout -k 10 400 python -u tools/commit_sweep.py 24 TPST_LIB_PATH=$R/testudo_amd/libtpst_m3.so > $OUT/ab_k1.txt 2>&1 || exit 1
timeout -k 10 400 python -u tools/commit_sweep.py 24 TPST_LIB_PATH=$R/testudo_amd/libtpst_m3.so >> $OUT/ab_k1.txt 2>&1 || exit 1
