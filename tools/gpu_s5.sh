# session GPU run (r01 s5): tests, smoke, bench, rocprof of the bench, commit/open traces at 2^20 and 2^24
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/s5
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > $OUT/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu > $OUT/bench_prof.json 2> $OUT/prof.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/po20 -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_open.py 20 3 > $OUT/po20.txt 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/po24 -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_open.py 24 3 > $OUT/po24.txt 2>&1
