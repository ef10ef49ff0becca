# look-ahead stream priority default (6) vs off (0): open parity, PST benches
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-prio6}
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
PT="python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $PT -k "sqrt_pst or open or fullsize or mipp or rccl" > $OUT/t_main.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no-cpu --no-r1cs --no-groth16 --steps 5 > $OUT/bench6.json 2> $OUT/bench6.err || exit 1
TPST_OPEN_PRIO=0 timeout -k 10 400 python -u bench.py --no-cpu --no-r1cs --no-groth16 --steps 5 > $OUT/bench0.json 2> $OUT/bench0.err || exit 1
timeout -k 10 400 python -u bench.py --no-cpu --no-r1cs --no-groth16 --steps 5 > $OUT/bench6b.json 2> $OUT/bench6b.err
