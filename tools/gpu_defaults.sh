# re-check of a few defaults on the final tree: open / commit sweeps at 2^20
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-defaults}
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
timeout -k 10 500 python -u tools/open_sweep.py 20 TPST_RNS_WG_PER_CU=1 TPST_INV_WAVE_MAX=0 TPST_OPEN_PRIO=6 TPST_AFFINE_BATCH=1 > $OUT/open20.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/commit_sweep.py 20 TPST_AFFINE_BATCH=1 TPST_INV_WAVE_MAX=0 > $OUT/commit20.txt 2>&1
