# full GPU test suite + microbenchmarks + bench (no CPU leg) + gather experiment
set -o pipefail
OUT=gpurun_out/${1:-r4b}
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
timeout -k 10 120 python -u tools/mb_fq29.py > $OUT/mb_fq29.log 2>&1 && \
timeout -k 10 60 python -u -c "
import sys; sys.path.insert(0, '.')
from testudo_amd import Context
ctx = Context(0)
ctx.microbench(2, 64, 2)
print('inv lone-wave us', min(ctx.microbench(2, 64, 20) for _ in range(3)) * 1e3 / 20, flush=True)
" >> $OUT/mb_fq29.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/gpu_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err && \
TPST_GATHER_MASK=12 timeout -k 10 300 python -u bench.py --no-cpu --no-pst --no-r1cs --no-groth16 --steps 5 > $OUT/gmask12.json 2> $OUT/gmask12.err
