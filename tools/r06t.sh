set -e
O=gpurun_out/r06t; mkdir -p $O
timeout -k 10 600 python3 tools/ab_bench.py --crc --rounds 5 base ECAMD_CRC_V=4 ECAMD_CRC_V=6 ECAMD_CRC_V=5 ECAMD_CRC_V=4,ECAMD_CRC_R=4 > $O/ab_crc.txt 2>&1
tail -6 $O/ab_crc.txt
timeout -k 10 400 python3 tools/ab_bench.py --rounds 5 base > $O/ab_plain.txt 2>&1
tail -2 $O/ab_plain.txt
