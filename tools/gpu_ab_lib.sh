# A/B: the default build (Pornin-form wave inverse) against libtpst_by.so
# (Bernstein-Yang form) and the chain-priority / batched-affine switches:
# parity subset, open and commit sweeps at 2^20: tools/gpu_ab_lib.sh TAG
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-ablib}
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
BY=$GRAFT_REPO_ROOT/testudo_amd/libtpst_by.so
PT="python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu"
TPST_AFFINE_BATCH=1 timeout -k 10 300 $PT -k "fq_inverse or sqrt_pst or multi_pairing or commit_rows" > $OUT/t_main.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/open_sweep.py 20 TPST_CHAIN_PRIO=2 TPST_AFFINE_BATCH=1 TPST_LIB_PATH=$BY,TPST_CHAIN_PRIO=0,TPST_AFFINE_BATCH=0 > $OUT/open20.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/commit_sweep.py 20 TPST_AFFINE_BATCH=1 TPST_LIB_PATH=$BY > $OUT/commit20.txt 2>&1
