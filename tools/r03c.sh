set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c; mkdir -p $O
V="base ECAMD_ENC_NOCOMP=1 ECAMD_DEC_NOCOMP=1 ECAMD_ENC_NTL=1 ECAMD_ENC_NTL=1,ECAMD_ENC_PER_CU=2 ECAMD_ENC_PER_CU=4"
timeout -k 10 300 python3 tools/ab_bench.py $V > $O/ab_b2b.txt 2>&1; cat $O/ab_b2b.txt
timeout -k 10 300 python3 tools/ab_bench.py --alt $V > $O/ab_alt.txt 2>&1; cat $O/ab_alt.txt
timeout -k 10 300 python3 tools/ab_bench.py --alt --flush-mb 512 base ECAMD_ENC_NTL=1 > $O/ab_alt_flush.txt 2>&1; cat $O/ab_alt_flush.txt
timeout -k 10 300 python3 tools/ab_bench.py --alt --crc base ECAMD_CRC_NTL=1 ECAMD_CRC_PER_CU=6 ECAMD_CRC_PER_CU=4 > $O/ab_crc.txt 2>&1; cat $O/ab_crc.txt
