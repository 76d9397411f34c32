set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03m; mkdir -p $O
timeout -k 10 300 python3 tools/ab_bench.py --alt --crc base ECAMD_CRC_RUN=0 > $O/ab_crc.txt 2>&1; cat $O/ab_crc.txt
timeout -k 10 300 python3 tools/ab_bench.py --alt --crc --bench-alloc base ECAMD_CRC_RUN=0 > $O/ab_crc_ba.txt 2>&1; cat $O/ab_crc_ba.txt
timeout -k 10 300 python3 tools/ab_bench.py --alt --bench-alloc base > $O/ab_ba.txt 2>&1; cat $O/ab_ba.txt
