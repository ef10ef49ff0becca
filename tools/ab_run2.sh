set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6e
mkdir -p $OUT
cd $R
bash tools/gpu_run.sh r6e tests bench valu prof || exit 1
cd $R && TPST_BENCH_SHARED_GPU=1 timeout -k 10 900 python -u bench.py --gpus 8 --no-cpu --steps 5 --warmup 2 > $OUT/bench_n8_shared.json 2> $OUT/bench_n8_shared.err || exit 1
