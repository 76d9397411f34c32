set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03x; mkdir -p $O
timeout -k 10 300 python3 tools/ab_bench.py --alt --rounds 10 base ECAMD_ENC_NTL=1 > $O/ab_alt.txt 2>&1; cat $O/ab_alt.txt
timeout -k 10 300 python3 tools/ab_bench.py --rounds 10 base ECAMD_ENC_NTL=1 > $O/ab_b2b.txt 2>&1; cat $O/ab_b2b.txt
timeout -k 10 300 python3 tools/ab_bench.py --alt --rounds 6 --k 6 --m 3 base ECAMD_ENC_NTL=1 > $O/ab_k6.txt 2>&1; tail -3 $O/ab_k6.txt
