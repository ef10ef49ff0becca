# stream placement A/B for the odd-round h preparation: default (stream A) vs
# TPST_OPEN_C=la; per-round traces and PST benches: tools/gpu_openc.sh TAG
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-openc}
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
PT="python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu"
TPST_OPEN_C=la timeout -k 10 600 $PT -k "open or fullsize or mipp" > $OUT/gpu_tests_la.log 2>&1 || exit 1
TPST_OPEN_TRACE=1 timeout -k 10 120 python -u tools/prof_open.py 20 3 > $OUT/trace_a_stdout.txt 2> $OUT/trace_a.txt || exit 1
TPST_OPEN_C=la TPST_OPEN_TRACE=1 timeout -k 10 120 python -u tools/prof_open.py 20 3 > $OUT/trace_la_stdout.txt 2> $OUT/trace_la.txt || exit 1
timeout -k 10 400 python -u bench.py --no-cpu --no-r1cs --no-groth16 --steps 5 > $OUT/bench_a.json 2> $OUT/bench_a.err || exit 1
TPST_OPEN_C=la timeout -k 10 400 python -u bench.py --no-cpu --no-r1cs --no-groth16 --steps 5 > $OUT/bench_la.json 2> $OUT/bench_la.err
