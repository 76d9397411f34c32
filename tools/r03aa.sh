set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03aa; mkdir -p $O
V="base ECAMD_DEC_NB=2 ECAMD_DEC_NB=2,ECAMD_DEC_PER_CU=3 ECAMD_DEC_NB=2,ECAMD_DEC_PER_CU=4 ECAMD_DEC_PER_CU=1 ECAMD_DEC_NB=10,ECAMD_DEC_PER_CU=1"
timeout -k 10 300 python3 tools/ab_bench.py --alt $V > $O/ab_alt.txt 2>&1; cat $O/ab_alt.txt
