# MSM GPU tests, then a bench sweep over "GROUPS:LG:RED2:SPLIT:PRIO[:FIXUPQUAD]" tuples (MSM only)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-sw}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
if [ -n "$3" ]; then
  timeout -k 10 300 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu -k "$3" > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
  tail -2 $OUT/gpu_tests.log
fi
for p in $2; do
  IFS=: read g l r sp pr fq <<< "$p"
  fq=${fq:-1}
  TPST_MSM_GROUPS=$g TPST_MSM_LG=$l TPST_MSM_RED2=$r TPST_MSM_SPLIT=$sp TPST_MSM_PRIO=$pr TPST_MSM_FIXUP_QUAD=$fq timeout -k 10 200 python -u bench.py --no-cpu --no-pst --no-sharded --no-r1cs --no-groth16 > $OUT/bench_${g}_${l}_${r}_${sp}_${pr}_${fq}.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/bench_${g}_${l}_${r}_${sp}_${pr}_${fq}.json')); print('g $g lg $l red2 $r split $sp prio $pr fq $fq', d['value'], d['ms_per_step'], d['stages_ms_per_step'], d['parity_ok'])"
done
