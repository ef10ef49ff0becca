# look-ahead 1 against h^(1) prepared in round 1 (TPST_LA1_OWN_H=1, E = 1)
# instead of h^(0) (E = 2): the GPU suite under the switch, then an
# interleaved commit + open A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r6ag}
mkdir -p $OUT
cd $R
TPST_LA1_OWN_H=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_la1.log 2>&1 || exit 1
for i in 1 2; do
for L in 0 1; do
TPST_LA1_OWN_H=$L timeout -k 10 300 python -u tools/prof_open.py 20 5 > $OUT/t20_la${L}_$i.txt 2>&1 || exit 1
TPST_LA1_OWN_H=$L timeout -k 10 300 python -u tools/prof_open.py 24 3 > $OUT/t24_la${L}_$i.txt 2>&1 || exit 1
done
done
