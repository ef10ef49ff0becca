# commit + open at 2^24 / 2^20 with the fold table built by the commit (default) or by the opening
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r6j}
mkdir -p $OUT
cd $R
for i in 1 2; do
timeout -k 10 300 python -u tools/prof_open.py 24 4 > $OUT/t24_default_$i.txt 2>&1 || exit 1
TPST_COMMIT_TABLE=0 timeout -k 10 300 python -u tools/prof_open.py 24 4 > $OUT/t24_notable_$i.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/prof_open.py 20 5 > $OUT/t20_default_$i.txt 2>&1 || exit 1
TPST_COMMIT_TABLE=0 timeout -k 10 300 python -u tools/prof_open.py 20 5 > $OUT/t20_notable_$i.txt 2>&1 || exit 1
done
