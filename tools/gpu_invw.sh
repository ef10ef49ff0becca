# wave-cooperative Fq inverse: parity, microbench, then MSM/open parity and
# the open trace: tools/gpu_invw.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-invw}
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
PT="python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 200 $PT -k "fq_inverse" > $OUT/t_inv.log 2>&1 || exit $?
timeout -k 10 120 python -u - > $OUT/mb_inv.log 2>&1 <<'PY' || exit $?
from testudo_amd import Context
c = Context(0)
for kind, threads, iters in [(2, 64, 20), (2, 1024, 20), (2, 65536, 20), (15, 64, 20), (15, 1024, 20), (15, 16384, 20), (15, 65536, 20)]:
    c.microbench(kind, threads, iters)
    ms = min(c.microbench(kind, threads, iters) for _ in range(3))
    print("kind %d threads %d: %.3f us per chain step" % (kind, threads, ms * 1e3 / iters), flush=True)
PY
timeout -k 10 600 $PT -k "msm or open or commit or verify or pairing" > $OUT/gpu_tests.log 2>&1 && \
TPST_OPEN_TRACE=1 timeout -k 10 400 python -u bench.py --no-cpu --no-r1cs --no-groth16 --no-sharded --steps 5 > $OUT/bench.json 2> $OUT/bench.err && \
TPST_INV_WAVE_MAX=0 timeout -k 10 400 python -u bench.py --no-cpu --no-r1cs --no-groth16 --no-sharded --steps 5 > $OUT/bench_lane.json 2> $OUT/bench_lane.err
