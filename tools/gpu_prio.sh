# wave inverse parity + timing, per-round trace, open priority sweep at 2^20:
# tools/gpu_prio.sh TAG
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-prio}
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
PT="python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 300 $PT -k "fq_inverse or golden or multi_pairing or g1_msm_vs_oracle" > $OUT/t_inv.log 2>&1 || exit 1
timeout -k 10 120 python -u - > $OUT/mb_inv.log 2>&1 <<'PY' || exit 1
from testudo_amd import Context
c = Context(0)
for kind, threads, iters in [(2, 64, 20), (15, 64, 20), (15, 16384, 20)]:
    c.microbench(kind, threads, iters)
    ms = min(c.microbench(kind, threads, iters) for _ in range(3))
    print("kind %d threads %d: %.3f us per chain step" % (kind, threads, ms * 1e3 / iters), flush=True)
PY
TPST_OPEN_TRACE=1 timeout -k 10 120 python -u tools/prof_open.py 20 3 > $OUT/trace_stdout.txt 2> $OUT/trace.txt || exit 1
timeout -k 10 500 python -u tools/open_sweep.py 20 TPST_CHAIN_PRIO=0 TPST_CHAIN_PRIO=3 TPST_OPEN_PRIO=6 TPST_OPEN_PRIO=7 > $OUT/sweep20.txt 2>&1
