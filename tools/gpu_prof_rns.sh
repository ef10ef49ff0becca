# kernel traces of sqrt-PST commit + open at 2^20 and 2^24 (tools/prof_open.py):
#   bash tools/gpu_prof_rns.sh TAG
set -o pipefail
TAG=${1:-profrns}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_open20 -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_open.py 20 3 > $OUT/prof_open20.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_open24 -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_open.py 24 3 > $OUT/prof_open24.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
for n in 20 24; do
  f=$(ls $OUT/prof_open$n/*/run_kernel_trace.csv 2>/dev/null | head -1)
  [ -z "$f" ] && f=$(ls $OUT/prof_open$n/run_kernel_trace.csv 2>/dev/null | head -1)
  python tools/open_timeline.py $f 600 > $OUT/open${n}_timeline.txt 2>&1
done
