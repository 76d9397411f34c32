set -e
O=gpurun_out/r06v; mkdir -p $O
timeout -k 10 600 python3 tools/ab_bench.py --crc --rounds 5 base ECAMD_CRC_V=7 ECAMD_CRC_V=8 ECAMD_CRC_V=10 > $O/ab_crc.txt 2>&1
tail -5 $O/ab_crc.txt
timeout -k 10 400 python3 tools/ab_bench.py --rounds 5 base > $O/ab_plain.txt 2>&1
tail -2 $O/ab_plain.txt
