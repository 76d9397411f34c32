set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03z; mkdir -p $O
V="base ECAMD_ENC_PAIR=3 ECAMD_ENC_PAIR=3,ECAMD_ENC_NTL=1 ECAMD_ENC_PAIR=5 ECAMD_ENC_PAIR=2 ECAMD_ENC_PAIR=3,ECAMD_ENC_PER_CU=3 ECAMD_ENC_PAIR=3,ECAMD_ENC_NTL=1,ECAMD_ENC_PER_CU=3"
timeout -k 10 300 python3 tools/ab_bench.py --alt $V > $O/ab_alt.txt 2>&1; cat $O/ab_alt.txt
MB_RANDOM=1 timeout -k 10 200 tools/membench 10 wpb > $O/membench_wpb.txt 2>&1; grep -E "wpb4 ld-nt  |wpb4   |pairs NP3 ld-nt" $O/membench_wpb.txt
