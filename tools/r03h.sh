set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03h; mkdir -p $O
V="base ECAMD_ENC_PER_CU=2 ECAMD_ENC_PER_CU=3 ECAMD_ENC_PER_CU=4"
for k in 2 4 6 8 12 7; do
  timeout -k 10 200 python3 tools/ab_bench.py --alt --rounds 3 --k $k --m 4 $V > $O/ab_k$k.txt 2>&1; cat $O/ab_k$k.txt | tail -5
done
timeout -k 10 200 python3 tools/ab_bench.py --alt --rounds 3 --k 4 --m 2 $V > $O/ab_k4m2.txt 2>&1; tail -5 $O/ab_k4m2.txt
timeout -k 10 200 python3 tools/ab_bench.py --alt --rounds 3 --ec-type isa_l_rs_cauchy --k 12 --m 4 --obj-bytes 16777216 --batch 128 $V > $O/ab_cauchy.txt 2>&1; tail -5 $O/ab_cauchy.txt
timeout -k 10 200 python3 tools/ab_bench.py --alt --rounds 3 --ec-type isa_l_rs_vand --k 10 --m 4 $V > $O/ab_isal10.txt 2>&1; tail -5 $O/ab_isal10.txt
