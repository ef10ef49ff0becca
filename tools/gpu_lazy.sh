# host Poseidon lazy reduction: box-CPU bench, open parity, per-round trace, PST bench
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-lazy}
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
./tools/bin/host_poseidon_bench > $OUT/poseidon_cpp.txt 2>&1 || exit 1
PT="python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $PT -k "sqrt_pst or open or fullsize or verify or transcript" > $OUT/t_main.log 2>&1 || exit 1
TPST_OPEN_TRACE=1 timeout -k 10 120 python -u tools/prof_open.py 20 3 > $OUT/trace_stdout.txt 2> $OUT/trace.txt || exit 1
timeout -k 10 400 python -u bench.py --no-cpu --no-r1cs --no-groth16 --steps 5 > $OUT/bench.json 2> $OUT/bench.err
