set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03g; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; tail -3 $O/pytest_gpu.log
V="base ECAMD_EDGE_BLOCKS=0 ECAMD_ENC_PER_CU=2 ECAMD_ENC_PER_CU=2,ECAMD_EDGE_BLOCKS=0 ECAMD_ENC_NTL=1,ECAMD_ENC_PER_CU=2 ECAMD_ENC_NOCOMP=1,ECAMD_ENC_PER_CU=2 ECAMD_DEC_NOCOMP=1 ECAMD_DEC_PER_CU=3"
timeout -k 10 300 python3 tools/ab_bench.py --alt $V > $O/ab_alt.txt 2>&1; cat $O/ab_alt.txt
timeout -k 10 300 python3 tools/ab_bench.py --alt --crc base ECAMD_EDGE_BLOCKS=0 ECAMD_CRC_NTL=1,ECAMD_CRC_PER_CU=2 ECAMD_CRC_PER_CU=2 > $O/ab_crc.txt 2>&1; cat $O/ab_crc.txt
