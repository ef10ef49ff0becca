# opening with A (t combination) and B (u-side MSM) on a reserved CU set of
# K CUs (TPST_OPEN_CUMASK=K), look-aheads and C on the rest; interleaved
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r6p}
mkdir -p $OUT
cd $R
for i in 1 2; do
for K in 0 32 64 96; do
TPST_OPEN_CUMASK=$K timeout -k 10 300 python -u tools/prof_open.py 20 5 > $OUT/t20_k${K}_$i.txt 2>&1 || exit 1
TPST_OPEN_CUMASK=$K timeout -k 10 300 python -u tools/prof_open.py 24 3 > $OUT/t24_k${K}_$i.txt 2>&1 || exit 1
done
done
