# K1 level-1 reduction segment length / form at 2^20 and 2^24 (commit + open,
# interleaved), kernel stats at 2^20 per setting, parity under the last one
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r6aa}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
SETS="lg4:TPST_K1_RED_LG=4 lg3:TPST_K1_RED_LG=3 lg2:TPST_K1_RED_LG=2 lg2l:TPST_K1_RED_LG=2,TPST_K1_RED_LANE=1"
for i in 1 2; do
for sp in $SETS; do
lab=${sp%%:*}; envs=${sp#*:}; envs=${envs//,/ }
env $envs timeout -k 10 300 python -u tools/prof_open.py 20 5 > $OUT/t20_${lab}_$i.txt 2>&1 || exit 1
env $envs timeout -k 10 300 python -u tools/prof_open.py 24 3 > $OUT/t24_${lab}_$i.txt 2>&1 || exit 1
done
done
for sp in $SETS; do
lab=${sp%%:*}; envs=${sp#*:}; envs=${envs//,/ }
cd /tmp && env $envs timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$lab -o run -- python3 $R/tools/prof_open.py 20 2 > $OUT/prof_$lab.log 2>&1 || exit 1
done
cd $R
for sp in lg3:TPST_K1_RED_LG=3 lg2l:TPST_K1_RED_LG=2,TPST_K1_RED_LANE=1; do
lab=${sp%%:*}; envs=${sp#*:}; envs=${envs//,/ }
env $envs timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_fullsize.py tests/test_boundary.py -x -q --timeout 300 --timeout-method thread -k "sqrt_pst or fullsize_commit_open or batch" > $OUT/tests_$lab.log 2>&1 || exit 1
done
