# K1 A/B: kernel stats of the 2^24 commit leg with the Edwards tables and with
# the Weierstrass tables (TPST_K1_XYZZ=1)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-k1ab}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="$GRAFT_REPO_ROOT/bench.py --no-cpu --no-pst --no-r1cs --no-groth16 --steps 3 --warmup 1"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ted -o run -- python3 $ARGS > $OUT/ted.json 2> $OUT/ted.err || exit 1
TPST_K1_XYZZ=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/xyzz -o run -- python3 $ARGS > $OUT/xyzz.json 2> $OUT/xyzz.err || exit 1
for v in ted xyzz; do echo "== $v"; python3 -c "
import csv,sys
r=list(csv.DictReader(open('$OUT/$v/run_kernel_stats.csv')))
for x in r[:12]: print('%10.3f ms %5s  %s' % (float(x['TotalDurationNs'])/1e6, x['Calls'], x['Name'][:110]))
"; done
