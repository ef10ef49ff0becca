# accumulation occupancy sweep: TPST_ACC_MINW (K2) and TPST_K1_MINW (K1)
set -o pipefail
OUT=gpurun_out/${1:-minw}
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
for w in 2 3 4; do
  TPST_ACC_MINW=$w timeout -k 10 200 python -u bench.py --no-cpu --no-pst --no-sharded --no-r1cs --no-groth16 > $OUT/msm_w$w.json 2> $OUT/msm_w$w.err || exit 1
done
for w in 2 3; do
  TPST_K1_MINW=$w timeout -k 10 300 python -u bench.py --no-cpu --no-pst --no-r1cs --no-groth16 --steps 3 > $OUT/k1_w$w.json 2> $OUT/k1_w$w.err || exit 1
done
