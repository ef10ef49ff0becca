# MSM tests on the current build, then an interleaved MSM A/B of libraries
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r6h}
shift
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "msm" > $OUT/msm_tests.log 2>&1 || exit 1
timeout -k 10 900 python -u tools/ab_libs.py 3 "$@" > $OUT/ab_msm.jsonl 2> $OUT/ab_msm.err || exit 1
