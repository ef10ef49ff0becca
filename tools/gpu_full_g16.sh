# full GPU suite, then the Groth16 bench leg and its profile
#   bash tools/gpu_full_g16.sh TAG
set -o pipefail
TAG=${1:-f}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -u bench.py --no-cpu --no-pst --no-sharded --no-r1cs --steps 3 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['groth16'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_g16.py 20 3 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
grep prove_s $OUT/prof.log
