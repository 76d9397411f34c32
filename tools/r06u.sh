set -e
O=gpurun_out/r06u; mkdir -p $O
timeout -k 10 500 python3 tools/ab_bench.py --rounds 7 base ECAMD_ENC_CV0=1 > $O/ab_plain.txt 2>&1
tail -3 $O/ab_plain.txt
timeout -k 10 500 python3 tools/ab_bench.py --full-stripe --rounds 5 base ECAMD_ENC_CV0=1 > $O/ab_full.txt 2>&1
tail -3 $O/ab_full.txt
timeout -k 10 500 python3 tools/ab_bench.py --crc --rounds 5 base ECAMD_CRC_V=10 ECAMD_CRC_V=4 > $O/ab_crc.txt 2>&1
tail -4 $O/ab_crc.txt
