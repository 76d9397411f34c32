set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03ah; mkdir -p $O
timeout -k 10 300 python3 tools/ab_bench.py --alt --crc --rounds 8 base ECAMD_CRC_DEFER=1 > $O/ab_crc.txt 2>&1; cat $O/ab_crc.txt
ECAMD_CRC_DEFER=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_edges.py -k crc -q --timeout 200 --timeout-method thread > $O/pytest_defer.log 2>&1; tail -2 $O/pytest_defer.log
