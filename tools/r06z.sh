set -e
O=gpurun_out/r06z; mkdir -p $O
timeout -k 10 600 python3 tools/ab_bench.py --crc --full-stripe --rounds 5 base ECAMD_ENC_DATA_W=12,ECAMD_ENC_DATA_R=3 ECAMD_ENC_DATA_W=12,ECAMD_ENC_DATA_R=4 ECAMD_ENC_DATA_W=16,ECAMD_ENC_DATA_R=3 > $O/ab_full_crc.txt 2>&1
tail -5 $O/ab_full_crc.txt
