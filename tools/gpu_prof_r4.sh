# Round-4 profiles: kernel traces (MSM, 2^20 / 2^24 commit + open), PMC passes
# (one counter group per run) of the MSM bench and of the 2^24 commit (K1).
#   bash tools/gpu_prof_r4.sh TAG
set -o pipefail
TAG=${1:-prof}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
SHORT="$GRAFT_REPO_ROOT/bench.py --no-cpu --no-pst --no-sharded --no-r1cs --no-groth16 --steps 5 --warmup 2"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_msm -o run -- python3 $SHORT > $OUT/prof_msm.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_open20 -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_open.py 20 3 > $OUT/prof_open20.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_open24 -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_open.py 24 3 > $OUT/prof_open24.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $SHORT > $OUT/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $SHORT > $OUT/pmc_write.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d $OUT/pmc_valu -o run -- python3 $SHORT > $OUT/pmc_valu.log 2>&1 || exit 1
K1="$GRAFT_REPO_ROOT/tools/prof_open.py 24 1"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/k1_fetch -o run -- python3 $K1 > $OUT/k1_fetch.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/k1_write -o run -- python3 $K1 > $OUT/k1_write.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d $OUT/k1_valu -o run -- python3 $K1 > $OUT/k1_valu.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/pmc_summary.py $OUT/pmc_bucket_acc_short.json $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_valu $OUT/prof_msm > $OUT/pmc_summary.log 2>&1
cd $GRAFT_REPO_ROOT && python tools/pmc_k1.py $OUT/pmc_bucket_acc_chunk_2p24.json $OUT/k1_fetch $OUT/k1_write $OUT/k1_valu $OUT/prof_open24 > $OUT/pmc_k1.log 2>&1
