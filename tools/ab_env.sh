# interleaved commit + open A/B over environment settings of one library:
#   bash tools/ab_env.sh OUT_TAG PASSES label1=VAR=val[,VAR=val] label2=... 
# then the opening parity tests under the last setting
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
PASSES=$2
shift 2
mkdir -p $OUT
cd $R
last=""
for i in $(seq 1 $PASSES); do
for spec in "$@"; do
lab=${spec%%=*}
envs=${spec#*=}
envs=${envs//,/ }
env $envs timeout -k 10 300 python -u tools/prof_open.py 20 5 > $OUT/t20_${lab}_$i.txt 2>&1 || exit 1
env $envs timeout -k 10 300 python -u tools/prof_open.py 24 3 > $OUT/t24_${lab}_$i.txt 2>&1 || exit 1
last=$envs
done
done
env $last timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_fullsize.py tests/test_sharded_open.py -x -q --timeout 300 --timeout-method thread -k "sqrt_pst or fullsize_commit_open or 11-2 or 12-4 or 13-8" > $OUT/open_tests.log 2>&1 || exit 1
