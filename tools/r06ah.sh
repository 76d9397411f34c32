set -e
O=gpurun_out/r06ah; mkdir -p $O
timeout -k 10 600 python3 tools/ab_bench.py --alt --rounds 7 base ECAMD_PRIO=1 > $O/ab_prio.txt 2>&1
tail -3 $O/ab_prio.txt
timeout -k 10 600 python3 tools/ab_bench.py --rounds 7 base ECAMD_PRIO=1 > $O/ab_prio_b2b.txt 2>&1
tail -3 $O/ab_prio_b2b.txt
