set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03e; mkdir -p $O
timeout -k 10 200 tools/membench 10 enc > $O/membench_const.txt 2>&1; tail -3 $O/membench_const.txt
MB_RANDOM=1 timeout -k 10 200 tools/membench 10 enc > $O/membench_rand.txt 2>&1; tail -3 $O/membench_rand.txt
V="base ECAMD_ENC_NOCOMP=1,ECAMD_ENC_PER_CU=1,ECAMD_ENC_NTL=1 ECAMD_ENC_NOCOMP=1,ECAMD_ENC_PER_CU=2,ECAMD_ENC_NTL=1 ECAMD_ENC_NOCOMP=1,ECAMD_ENC_PER_CU=4,ECAMD_ENC_NTL=1 ECAMD_ENC_NOCOMP=1,ECAMD_ENC_NTL=1 ECAMD_ENC_NOCOMP=1,ECAMD_ENC_PER_CU=2 ECAMD_ENC_NTL=1,ECAMD_ENC_PER_CU=2"
timeout -k 10 300 python3 tools/ab_bench.py $V > $O/ab_b2b.txt 2>&1; cat $O/ab_b2b.txt
timeout -k 10 300 python3 tools/ab_bench.py --alt --crc base ECAMD_CRC_NTL=1,ECAMD_CRC_PER_CU=2 ECAMD_CRC_NTL=1,ECAMD_CRC_PER_CU=3 ECAMD_CRC_NTL=1,ECAMD_CRC_PER_CU=4 ECAMD_CRC_NTL=1,ECAMD_CRC_PER_CU=6 ECAMD_CRC_NTL=1 > $O/ab_crc.txt 2>&1; cat $O/ab_crc.txt
