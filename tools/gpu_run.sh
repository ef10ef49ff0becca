# GPU-box session steps (run through gpurun from the repo root):
#   bash tools/gpu_run.sh TAG step [step ...]
# steps:
#   tests   pytest -m gpu + smoke
#   msmtests  only the MSM tests of tests/test_gpu.py
#   bench   default bench.py (JSON line -> bench.json)
#   prof    rocprofv3 kernel traces + stats: MSM bench, 2^20 and 2^24 commit+open
#   pmc     PMC passes (FETCH_SIZE, WRITE_SIZE, VALU, stall counters) on the MSM bench
#   k1pmc   PMC passes (FETCH_SIZE, WRITE_SIZE, VALU) on the 2^24 commit (K1)
#   solo    per-rank latency of the sharded opening (tools/shard_open_solo.py, W = 2/4/8)
#   valu    VALU slots / busy / divergence PMC pass of K2 (MSM bench) and K1 (2^24 commit)
#   icache  instruction-cache PMC pass of the MSM bench
#   list    rocprofv3 -L (available counters)
# Every GPU step runs under its own time limit; the first failure ends the script.
set -o pipefail
TAG=${1:-run}
shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
R=$GRAFT_REPO_ROOT
SHORT="$R/bench.py --no-cpu --no-pst --no-sharded --no-r1cs --no-groth16 --steps 5 --warmup 2"
K1="$R/tools/prof_open.py 24 1"
export TMPDIR=/tmp
for step in "$@"; do
  echo "[gpu_run] $step $(date +%T)"
  case $step in
    tests)
      cd $R && timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/gpu_tests.log 2>&1 || exit 1
      cd $R && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1 ;;
    msmtests)
      cd $R && timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "msm" > $OUT/msm_tests.log 2>&1 || exit 1 ;;
    bench)
      cd $R && timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1 ;;
    prof)
      cd /tmp
      timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_msm -o run -- python3 $SHORT > $OUT/prof_msm.log 2>&1 || exit 1
      timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_open20 -o run -- python3 $R/tools/prof_open.py 20 3 > $OUT/prof_open20.log 2>&1 || exit 1
      timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_open24 -o run -- python3 $R/tools/prof_open.py 24 3 > $OUT/prof_open24.log 2>&1 || exit 1 ;;
    pmc)
      cd /tmp
      timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $SHORT > $OUT/pmc_fetch.log 2>&1 || exit 1
      timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $SHORT > $OUT/pmc_write.log 2>&1 || exit 1
      timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d $OUT/pmc_valu -o run -- python3 $SHORT > $OUT/pmc_valu.log 2>&1 || exit 1
      timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc_stall -o run -- python3 $SHORT > $OUT/pmc_stall.log 2>&1 || exit 1
      cd $R && python tools/pmc_summary.py $OUT/pmc_bucket_acc_short.json $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_valu $OUT/prof_msm > $OUT/pmc_summary.log 2>&1
      cd $R && python tools/pmc_stall.py $OUT/pmc_stall.json $OUT/pmc_stall > $OUT/pmc_stall_summary.log 2>&1 ;;
    valu)
      cd /tmp
      timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_valu2 -o run -- python3 $SHORT > $OUT/pmc_valu2.log 2>&1 || exit 1
      cd $R && python tools/pmc_valu.py $OUT/pmc_valu_k2.json $OUT/pmc_valu2 k_bucket_acc_short 3 k_mb_fq29 > $OUT/pmc_valu_k2.log 2>&1
      cd /tmp
      timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/k1_valu2 -o run -- python3 $K1 > $OUT/k1_valu2.log 2>&1 || exit 1
      cd $R && python tools/pmc_valu.py $OUT/pmc_valu_k1.json $OUT/k1_valu2 k_bucket_acc_chunk_lds 1 > $OUT/pmc_valu_k1.log 2>&1 ;;
    icache)
      cd /tmp
      timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH --output-format csv -d $OUT/pmc_icache -o run -- python3 $SHORT > $OUT/pmc_icache.log 2>&1 || exit 1 ;;
    k1pmc)
      cd /tmp
      timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/k1_fetch -o run -- python3 $K1 > $OUT/k1_fetch.log 2>&1 || exit 1
      timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/k1_write -o run -- python3 $K1 > $OUT/k1_write.log 2>&1 || exit 1
      timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d $OUT/k1_valu -o run -- python3 $K1 > $OUT/k1_valu.log 2>&1 || exit 1
      cd $R && python tools/pmc_k1.py $OUT/pmc_bucket_acc_chunk_2p24.json $OUT/k1_fetch $OUT/k1_write $OUT/k1_valu $OUT/prof_open24 > $OUT/pmc_k1.log 2>&1
      cd /tmp
      timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_BUSY_CYCLES --output-format csv -d $OUT/k1_stall -o run -- python3 $K1 > $OUT/k1_stall.log 2>&1 || exit 1
      cd $R && python tools/pmc_stall.py $OUT/pmc_stall_k1.json $OUT/k1_stall k_bucket_acc_chunk_lds > $OUT/pmc_stall_k1_summary.log 2>&1 ;;
    solo)
      cd $R && for w in 2 4 8; do timeout -k 10 300 python -u tools/shard_open_solo.py 24 $w 5 >> $OUT/shard_open_solo.jsonl 2>> $OUT/shard_open_solo.err || exit 1; done
      cd $R && timeout -k 10 300 python -u tools/shard_open_solo.py 20 8 5 >> $OUT/shard_open_solo.jsonl 2>> $OUT/shard_open_solo.err || exit 1 ;;
    list)
      cd /tmp && timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || exit 1 ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[gpu_run] done $(date +%T)"
