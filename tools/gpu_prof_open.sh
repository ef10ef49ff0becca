# rocprofv3 kernel stats of sqrt-PST commit+open (tools/prof_open.py) at 2^$1
set -o pipefail
N=${1:-20}
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_open_$N
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_open.py $N 3 > $OUT/stdout.txt 2> $OUT/stderr.txt
