# opening A/B over runtime switches (host enqueue order, RNS wave priorities),
# interleaved, then the opening parity tests with every switch on
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r6o}
mkdir -p $OUT
cd $R
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 300 python -u tools/prof_open.py 20 5 > $OUT/t20_${lab}_$i.txt 2>&1 || return 1
  env "$@" timeout -k 10 300 python -u tools/prof_open.py 24 3 > $OUT/t24_${lab}_$i.txt 2>&1 || return 1
}
for i in 1 2; do
run base X=0 || exit 1
run afirst TPST_OPEN_A_FIRST=1 || exit 1
run cprio TPST_COMBINE_PRIO=3 || exit 1
run bothprio TPST_COMBINE_PRIO=3 TPST_CHAIN_PRIO=2 || exit 1
run all TPST_OPEN_A_FIRST=1 TPST_COMBINE_PRIO=3 TPST_CHAIN_PRIO=2 || exit 1
done
TPST_OPEN_A_FIRST=1 TPST_COMBINE_PRIO=3 TPST_CHAIN_PRIO=2 timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_fullsize.py tests/test_sharded_open.py -x -q --timeout 300 --timeout-method thread -k "sqrt_pst or fullsize_commit_open or 11-2 or 12-4 or 13-8" > $OUT/open_tests_all.log 2>&1 || exit 1
