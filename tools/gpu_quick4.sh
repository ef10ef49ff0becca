# MSM / K1 parity tests + the bench without the CPU leg: tools/gpu_quick4.sh TAG [pytest -k expr]
set -o pipefail
OUT=gpurun_out/${1:-q4}
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
K=${2:-"msm or commit or fullsize or split or pairing or open"}
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu -k "$K" > $OUT/gpu_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err && \
  TPST_GATHER_MASK=12 timeout -k 10 300 python -u bench.py --no-cpu --no-pst --no-r1cs --no-groth16 --steps 5 > $OUT/gmask12.json 2> $OUT/gmask12.err
# (last step: every gathered point index masked to 12 bits -- the same access
#  pattern over a 384 KB cache-resident slice; sums wrong, timing only)
