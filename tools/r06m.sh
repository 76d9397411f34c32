set -e
O=gpurun_out/r06m; mkdir -p $O
timeout -k 10 400 python3 tools/ab_bench.py --crc --rounds 5 base ECAMD_CRC_V=3 > $O/ab_crc.txt 2>&1
tail -3 $O/ab_crc.txt
timeout -k 10 400 python3 tools/ab_bench.py --rounds 5 base > $O/ab_plain.txt 2>&1
tail -2 $O/ab_plain.txt
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "crc" --timeout 300 --timeout-method thread > $O/pytest_crc.log 2>&1
tail -2 $O/pytest_crc.log
