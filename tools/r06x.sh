set -e
O=gpurun_out/r06x; mkdir -p $O
timeout -k 10 500 python3 tools/ab_bench.py --crc --rounds 7 base ECAMD_CRC_V=10 > $O/ab_crc.txt 2>&1
tail -3 $O/ab_crc.txt
timeout -k 10 500 python3 tools/ab_bench.py --rounds 7 base > $O/ab_plain.txt 2>&1
tail -2 $O/ab_plain.txt
timeout -k 10 500 python3 tools/ab_bench.py --crc --full-stripe --rounds 5 base > $O/ab_full_crc.txt 2>&1
tail -2 $O/ab_full_crc.txt
timeout -k 10 500 python3 tools/ab_bench.py --full-stripe --rounds 5 base > $O/ab_full.txt 2>&1
tail -2 $O/ab_full.txt
