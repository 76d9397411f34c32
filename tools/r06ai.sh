set -e
O=gpurun_out/r06ai; mkdir -p $O
timeout -k 10 60 ./tools/build/mfma_probe > $O/mfma_probe.txt 2>&1 || true
cat $O/mfma_probe.txt
timeout -k 10 600 python3 tools/ab_bench.py --crc --rounds 7 base ECAMD_CRC_V=7 > $O/ab_crc.txt 2>&1
tail -3 $O/ab_crc.txt
timeout -k 10 400 python3 tools/ab_bench.py --rounds 5 base > $O/ab_plain.txt 2>&1
tail -2 $O/ab_plain.txt
