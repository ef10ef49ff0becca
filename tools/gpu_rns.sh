# RNS pairing pipeline parity + open timing: tools/gpu_rns.sh TAG [pytest -k expr]
# quick pairing parity first; on an assertion failure (rc 1) the same tests
# with the radix-engine tree levels (TPST_TREE_RNS=0) to localize it
set -o pipefail
OUT=gpurun_out/${1:-rns}
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
PT="python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 300 $PT -k "multi_pairing or bilinearity" > $OUT/t_quick.log 2>&1
rc=$?
if [ $rc -ne 0 ]; then
  if [ $rc -eq 1 ]; then
    TPST_TREE_RNS=0 timeout -k 10 300 $PT -k "multi_pairing or bilinearity" > $OUT/t_notree.log 2>&1
  fi
  exit $rc
fi
K=${2:-"pairing or ipp or open or verify or mipp or gt or final or commit"}
timeout -k 10 600 $PT -k "$K" > $OUT/gpu_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py --no-cpu --no-r1cs --no-groth16 --steps 5 > $OUT/bench.json 2> $OUT/bench.err && \
TPST_CHAIN_RNS=0 timeout -k 10 400 python -u bench.py --no-cpu --no-r1cs --no-groth16 --no-sharded --steps 5 > $OUT/bench_old.json 2> $OUT/bench_old.err
