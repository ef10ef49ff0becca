# parity subset + per-round trace + sweeps (batched affine switch) + PST bench:
# tools/gpu_check5.sh TAG
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-check5}
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
PT="python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu"
TPST_AFFINE_BATCH=1 timeout -k 10 600 $PT -k "fq_inverse or golden or multi_pairing or sqrt_pst or commit or open or fullsize" > $OUT/t_main.log 2>&1 || exit 1
TPST_OPEN_TRACE=1 timeout -k 10 120 python -u tools/prof_open.py 20 3 > $OUT/trace_stdout.txt 2> $OUT/trace.txt || exit 1
timeout -k 10 400 python -u tools/open_sweep.py 20 TPST_AFFINE_BATCH=1 > $OUT/open20.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/commit_sweep.py 20 TPST_AFFINE_BATCH=1 > $OUT/commit20.txt 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no-cpu --no-r1cs --no-groth16 --steps 5 > $OUT/bench.json 2> $OUT/bench.err
