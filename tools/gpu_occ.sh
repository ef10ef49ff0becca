# k_line_pair occupancy A/B (TPST_LINE_OCC = 1 / 2 / 4): parity with 4, open
# sweeps at 2^20 and 2^24: tools/gpu_occ.sh TAG
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-occ}
cd $GRAFT_REPO_ROOT
mkdir -p $OUT
PT="python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu"
TPST_LINE_OCC=4 timeout -k 10 300 $PT -k "multi_pairing or sqrt_pst_golden or sqrt_pst_vs_cpu or pairing_bilinearity" > $OUT/t_occ4.log 2>&1 || exit 1
TPST_LINE_OCC=2 timeout -k 10 300 $PT -k "multi_pairing or sqrt_pst_golden" > $OUT/t_occ2.log 2>&1 || exit 1
timeout -k 10 500 python -u tools/open_sweep.py 20 TPST_LINE_OCC=2 TPST_LINE_OCC=4 > $OUT/open20.txt 2>&1 || exit 1
timeout -k 10 600 python -u tools/open_sweep.py 24 TPST_LINE_OCC=4 > $OUT/open24.txt 2>&1
