# A/B of the current build against the previous one (libtpst_prev.so): GPU
# tests on the current, the MSM bench and the 2^24 commit on both
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r6f}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/ab_libs.py 3 new=testudo_amd/libtpst.so prev=testudo_amd/libtpst_prev.so > $OUT/ab_msm.jsonl 2> $OUT/ab_msm.err || exit 1
timeout -k 10 400 python -u tools/commit_sweep.py 24 TPST_LIB_PATH=$R/testudo_amd/libtpst_prev.so > $OUT/ab_k1.txt 2>&1 || exit 1
timeout -k 10 400 python -u tools/commit_sweep.py 24 TPST_LIB_PATH=$R/testudo_amd/libtpst_prev.so >> $OUT/ab_k1.txt 2>&1 || exit 1
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_open20 -o run -- python3 $R/tools/prof_open.py 20 3 > $OUT/prof_open20.log 2>&1 || exit 1
cd $R && python tools/open_critical.py $OUT/prof_open20/run_kernel_trace.csv > $OUT/open20_critical.txt 2>&1
cd $R && TPST_OPEN_TRACE=1 timeout -k 10 240 python -u tools/prof_open.py 20 4 > $OUT/open20_trace.txt 2>&1 || exit 1
cd $R && TPST_LIB_PATH=$R/testudo_amd/libtpst_prev.so TPST_OPEN_TRACE=1 timeout -k 10 240 python -u tools/prof_open.py 20 4 > $OUT/open20_trace_prev.txt 2>&1 || exit 1
