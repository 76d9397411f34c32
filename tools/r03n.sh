set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03n; mkdir -p $O
B="--steps 10 --no-host --no-cpu-baseline --fresh-steps 2"
for v in "plain:" "plain_nonuma:--no-numa" "crc:--inline-crc32" "crc_nonuma:--inline-crc32 --no-numa"; do
  name=${v%%:*}; a=${v#*:}
  ECAMD_CRC_RUN=0 timeout -k 10 300 python3 bench.py $B $a > $O/bench_$name.json 2>/dev/null
  python3 -c "import json;d=json.load(open('$O/bench_$name.json'));print('$name', d['kernels']['encode']['ms'], d['kernels']['decode']['ms'], d['value'])"
done
ECAMD_CRC_RUN=0 timeout -k 10 300 python3 tools/ab_bench.py --alt --crc --bench-alloc base > $O/ab_crc.txt 2>&1; tail -2 $O/ab_crc.txt
timeout -k 10 300 python3 tools/ab_bench.py --alt --bench-alloc base > $O/ab.txt 2>&1; tail -2 $O/ab.txt
