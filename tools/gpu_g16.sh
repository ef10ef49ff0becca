# Groth16 iteration: its GPU tests, then the bench's Groth16 leg alone
#   bash tools/gpu_g16.sh TAG
set -o pipefail
TAG=${1:-g16}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_groth16.py -x -v --timeout 200 --timeout-method thread -m gpu > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python -u bench.py --no-cpu --no-pst --no-sharded --no-r1cs --steps 3 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['groth16'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python -u bench.py --no-cpu --no-pst --no-sharded --no-r1cs --steps 3 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
echo done
