set -e
O=gpurun_out/r06y; mkdir -p $O
timeout -k 10 500 python3 tools/ab_bench.py --crc --full-stripe --rounds 5 base ECAMD_CRC_V=10 > $O/ab_full_crc.txt 2>&1
tail -3 $O/ab_full_crc.txt
timeout -k 10 500 python3 tools/ab_bench.py --full-stripe --rounds 5 base > $O/ab_full.txt 2>&1
tail -2 $O/ab_full.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dma.py tests/test_gpu_api.py tests/test_gpu_configs.py -m gpu -x -q -k "crc" --timeout 300 --timeout-method thread > $O/pytest_crc.log 2>&1
tail -2 $O/pytest_crc.log
