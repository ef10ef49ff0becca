# open parity + host Poseidon timing on the box CPU + per-round open trace and
# bench at 2^20: tools/gpu_trace20.sh TAG
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-trace20}
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
PT="python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $PT -k "open or verify or mipp or fullsize or rccl" > $OUT/gpu_tests.log 2>&1 || exit 1
python -u tools/host_poseidon_bench.py > $OUT/poseidon.txt 2>&1 || exit 1
TPST_OPEN_TRACE=1 timeout -k 10 120 python -u tools/prof_open.py 20 3 > $OUT/open_trace_stdout.txt 2> $OUT/open_trace.txt || exit 1
timeout -k 10 400 python -u bench.py --no-cpu --no-r1cs --no-groth16 --steps 5 > $OUT/bench.json 2> $OUT/bench.err
./tools/bin/host_poseidon_bench > $OUT/poseidon_cpp.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_open20 -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_open.py 20 3 > $OUT/prof_open20.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/open_timeline.py $OUT/prof_open20/run_kernel_trace.csv 600 > $OUT/open20_timeline.txt 2>&1
