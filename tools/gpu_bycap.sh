# wave inverse with the 80-batch cap: parity subset + microbenchmark
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-bycap}
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
PT="python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $PT -k "fq_inverse or golden or multi_pairing or sqrt_pst or g1_msm or pairing_bilinearity" > $OUT/t_main.log 2>&1 || exit 1
timeout -k 10 120 python -u - > $OUT/mb_inv.log 2>&1 <<'PY'
from testudo_amd import Context
c = Context(0)
for kind, threads, iters in [(2, 64, 20), (15, 64, 20), (15, 16384, 20)]:
    c.microbench(kind, threads, iters)
    ms = min(c.microbench(kind, threads, iters) for _ in range(3))
    print("kind %d threads %d: %.3f us per chain step" % (kind, threads, ms * 1e3 / iters), flush=True)
PY
