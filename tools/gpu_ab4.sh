# A/B experiments: wave-engine phases, inversion latency, MSM variants
#   bash tools/gpu_ab4.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-ab4}
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
timeout -k 10 120 python -u tools/mb_wave.py > $OUT/mb_wave.log 2>&1 || exit 1
timeout -k 10 60 python -u -c "
import sys; sys.path.insert(0, '.')
from testudo_amd import Context
ctx = Context(0)
ctx.microbench(2, 64, 2)
print('inv lone-wave us', min(ctx.microbench(2, 64, 20) for _ in range(3)) * 1e3 / 20, flush=True)
" >> $OUT/mb_wave.log 2>&1 || exit 1
M="--no-cpu --no-pst --no-sharded --no-r1cs --no-groth16 --steps 20"
timeout -k 10 120 python -u bench.py $M > $OUT/msm_base.json 2>&1 || exit 1
TPST_ACC_LDS=1 timeout -k 10 120 python -u bench.py $M > $OUT/msm_lds2.json 2>&1 || exit 1
TPST_ACC_LDS=1 TPST_ACC_MINW=3 timeout -k 10 120 python -u bench.py $M > $OUT/msm_lds3.json 2>&1 || exit 1
TPST_MSM_RED2=2 timeout -k 10 120 python -u bench.py $M > $OUT/msm_red2.json 2>&1 || exit 1
TPST_MSM_LG=5 timeout -k 10 120 python -u bench.py $M > $OUT/msm_lg5.json 2>&1 || exit 1
