# the opening's fold table prebuilt in the commit: parity subset, commit /
# open sweeps (TPST_COMMIT_TABLE=0 = built in the open), PST bench
#   tools/gpu_table.sh TAG
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-table}
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
PT="python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $PT -k "sqrt_pst or open or fullsize or commit or verify" > $OUT/t_main.log 2>&1 || exit 1
TPST_OPEN_TRACE=1 timeout -k 10 120 python -u tools/prof_open.py 20 3 > $OUT/trace_stdout.txt 2> $OUT/trace.txt || exit 1
TPST_COMMIT_TABLE=0 timeout -k 10 120 python -u tools/prof_open.py 20 3 > $OUT/trace0_stdout.txt 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no-cpu --no-r1cs --no-groth16 --steps 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
TPST_COMMIT_TABLE=0 timeout -k 10 400 python -u bench.py --no-cpu --no-r1cs --no-groth16 --steps 5 > $OUT/bench0.json 2> $OUT/bench0.err
