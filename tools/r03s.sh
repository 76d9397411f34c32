set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03s; mkdir -p $O
V="base ECAMD_ENC_WIDE=1 ECAMD_ENC_WIDE=1,ECAMD_ENC_NTL=1 ECAMD_ENC_WIDE=1,ECAMD_ENC_PER_CU=3 ECAMD_ENC_NOCOMP=1"
timeout -k 10 300 python3 tools/ab_bench.py --alt $V > $O/ab_alt.txt 2>&1; cat $O/ab_alt.txt
MB_RANDOM=1 timeout -k 10 200 tools/membench 10 ceil > $O/membench_ceil.txt 2>&1; grep -E "bpc=2" $O/membench_ceil.txt
timeout -k 10 300 python3 tools/ab_bench.py --alt --crc base ECAMD_CRC_WIDE=1 ECAMD_CRC_WIDE=1,ECAMD_CRC_NTL=1 ECAMD_CRC_WIDE=1,ECAMD_CRC_PER_CU=3 > $O/ab_crc.txt 2>&1; cat $O/ab_crc.txt
