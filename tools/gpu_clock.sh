# GPU state check: clocks / power / temperature, Fq29 microbenchmark rate,
# MSM bench and the 2^20 open: tools/gpu_clock.sh TAG
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-clock}
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
rocm-smi --showclocks --showpower --showtemp --showuse > $OUT/smi_before.txt 2>&1
timeout -k 10 120 python -u tools/mb_fq29.py > $OUT/mb_fq29.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu --no-pst --no-sharded --no-r1cs --no-groth16 --steps 10 > $OUT/bench_msm.json 2> $OUT/bench_msm.err || exit 1
timeout -k 10 300 python -u tools/open_sweep.py 20 > $OUT/open20.txt 2>&1
rocm-smi --showclocks --showpower --showtemp --showuse > $OUT/smi_after.txt 2>&1
