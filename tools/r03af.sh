set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03af; mkdir -p $O
: > $O/sweep.txt
for km in "4 2" "6 3" "8 4" "10 4" "12 4" "16 4" "20 4" "10 2" "12 6"; do
  set -- $km
  timeout -k 10 200 python3 tools/ab_bench.py --alt --rounds 3 --k $1 --m $2 base 2>/dev/null | tail -1 | sed "s/^base/k=$1 m=$2/" >> $O/sweep.txt
done
for km in "12 4" "10 4" "8 3"; do
  set -- $km
  timeout -k 10 200 python3 tools/ab_bench.py --alt --rounds 3 --ec-type isa_l_rs_cauchy --k $1 --m $2 base 2>/dev/null | tail -1 | sed "s/^base/cauchy k=$1 m=$2/" >> $O/sweep.txt
done
cat $O/sweep.txt
