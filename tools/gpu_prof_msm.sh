# rocprofv3 kernel trace of the 2^20 MSM bench leg (tools/msm_timeline.py reads it)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_msm
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-pst --no-sharded --no-groth16 --no-r1cs --steps 5 --warmup 2 > $OUT/stdout.txt 2> $OUT/stderr.txt
