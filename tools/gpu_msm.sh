# MSM iteration: MSM GPU tests, bench per window-group count, primitive rates
#   bash tools/gpu_msm.sh TAG "groups..."
set -o pipefail
TAG=${1:-m}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu -k "msm or smoke" > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
for g in ${2:-4}; do
  TPST_MSM_GROUPS=$g timeout -k 10 200 python -u bench.py --no-cpu --no-pst --no-sharded > $OUT/bench_g$g.json 2> $OUT/bench_g$g.err || { tail -20 $OUT/bench_g$g.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/bench_g$g.json')); print('groups $g', d['value'], d['ms_per_step'], d['stages_ms_per_step'], d['parity_ok'])"
done
timeout -k 10 120 python -u tools/mb_ops.py > $OUT/mb_ops.log 2>&1 && cat $OUT/mb_ops.log
