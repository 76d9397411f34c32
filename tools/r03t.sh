set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03t; mkdir -p $O
C3="--ec-type isa_l_rs_cauchy --k 12 --m 4 --obj-bytes 16777216 --batch 128 --second reconstruct --steps 10 --no-host --no-cpu-baseline --fresh-steps 0"
for pc in 4 2 3 6; do
  ECAMD_REC_PER_CU=$pc timeout -k 10 300 python3 bench.py $C3 > $O/config3_rec$pc.json 2>/dev/null
  python3 -c "import json;d=json.load(open('$O/config3_rec$pc.json'));print('rec_per_cu=$pc', d['kernels'], d['value'], d['verified'])"
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_multirank.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_multirank.log 2>&1; tail -2 $O/pytest_multirank.log
