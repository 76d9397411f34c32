set -e
O=gpurun_out/r06ac; mkdir -p $O
timeout -k 10 600 python3 tools/ab_bench.py --full-stripe --rounds 7 base ECAMD_ENC_CV0=1 > $O/ab_full.txt 2>&1
tail -3 $O/ab_full.txt
timeout -k 10 600 python3 tools/ab_bench.py --rounds 7 base ECAMD_ENC_CV0=1 > $O/ab_plain.txt 2>&1
tail -3 $O/ab_plain.txt
