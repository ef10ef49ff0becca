# Round session on the GPU box: tests, smoke, bench, rocprofv3 kernel stats of
# the bench, PMC passes (one counter group per run) on a short bench.
#   bash tools/gpu_session.sh TAG [notests]
set -o pipefail
TAG=${1:-run}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
if [ "$2" != "notests" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/gpu_tests.log 2>&1 || exit 1
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
fi
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_msm -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-pst --no-sharded --no-r1cs --no-groth16 --steps 5 --warmup 2 > $OUT/prof_msm.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_open20 -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_open.py 20 3 > $OUT/prof_open20.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_open24 -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_open.py 24 3 > $OUT/prof_open24.log 2>&1 || exit 1
SHORT="$GRAFT_REPO_ROOT/bench.py --no-cpu --no-pst --no-sharded --no-r1cs --no-groth16 --steps 5 --warmup 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu > $OUT/bench_prof.json 2> $OUT/prof.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $SHORT > $OUT/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $SHORT > $OUT/pmc_write.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d $OUT/pmc_valu -o run -- python3 $SHORT > $OUT/pmc_valu.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/pmc_summary.py $OUT/pmc_bucket_acc_short.json $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_valu $OUT/prof_msm > $OUT/pmc_summary.log 2>&1
