# G1 window-size sweep of the 2^20 MSM bench leg (TPST_MSM_C), with its tests
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-msmc}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for c in ${2:-16 19 20 22}; do
  TPST_MSM_C=$c timeout -k 10 200 python -u bench.py --no-cpu --no-pst --no-sharded --no-r1cs --no-groth16 > $OUT/bench_c$c.json 2> $OUT/bench_c$c.err || { tail -20 $OUT/bench_c$c.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_c$c.json')); print('c $c', d['value'], d['ms_per_step'], d['stages_ms_per_step'], d['parity_ok'])"
done
