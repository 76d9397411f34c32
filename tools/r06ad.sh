set -e
O=gpurun_out/r06ad; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -2 $O/pytest_gpu.log
for km in "12 2" "12 4" "14 4" "10 4"; do set -- $km
  timeout -k 10 300 python3 tools/ab_bench.py --k $1 --m $2 --rounds 5 base ECAMD_ENC_AL0=1 > $O/ab_k$1_m$2.txt 2>&1
  echo "k=$1 m=$2"; tail -2 $O/ab_k$1_m$2.txt
done
timeout -k 10 300 python3 tools/ab_bench.py --full-stripe --k 12 --m 4 --rounds 5 base ECAMD_ENC_AL0=1 > $O/ab_full_k12.txt 2>&1
tail -2 $O/ab_full_k12.txt
