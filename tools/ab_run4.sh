# GPU tests + open A/B (current vs libtpst_prev.so): host trace and kernel-trace attribution
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r6g}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $OUT/gpu_tests.log 2>&1 || exit 1
./tools/bin/host_poseidon_bench > $OUT/host_poseidon_bench.txt 2>&1 || true
for i in 1 2; do
cd $R && TPST_OPEN_TRACE=1 timeout -k 10 240 python -u tools/prof_open.py 20 4 > $OUT/open20_trace_$i.txt 2>&1 || exit 1
cd $R && TPST_LIB_PATH=$R/testudo_amd/libtpst_prev.so TPST_OPEN_TRACE=1 timeout -k 10 240 python -u tools/prof_open.py 20 4 > $OUT/open20_trace_prev_$i.txt 2>&1 || exit 1
done
cd $R && TPST_OPEN_TRACE=1 timeout -k 10 240 python -u tools/prof_open.py 24 3 > $OUT/open24_trace.txt 2>&1 || exit 1
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_open20 -o run -- python3 $R/tools/prof_open.py 20 3 > $OUT/prof_open20.log 2>&1 || exit 1
cd $R && python tools/open_critical.py $OUT/prof_open20/run_kernel_trace.csv > $OUT/open20_critical.txt 2>&1
