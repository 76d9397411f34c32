set -e
O=gpurun_out/r06j; mkdir -p $O
timeout -k 10 300 python3 tools/ab_bench.py --full-stripe --rounds 5 base ECAMD_XCD=0 > $O/ab_full_xcd.txt 2>&1
tail -3 $O/ab_full_xcd.txt
for km in "12 2" "6 2" "4 2" "10 1" "8 4" "12 4"; do
  set -- $km
  timeout -k 10 300 python3 tools/ab_bench.py --k $1 --m $2 --rounds 3 base ECAMD_ENC_STREAM2=1 > $O/ab_k$1_m$2.txt 2>&1
  tail -3 $O/ab_k$1_m$2.txt
done
