set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03q; mkdir -p $O
MB_RANDOM=1 timeout -k 10 200 tools/membench 10 ceil > $O/membench_ceil.txt 2>&1; grep -E "bpc=2" $O/membench_ceil.txt
B="--steps 20 --no-host --no-cpu-baseline --fresh-steps 2"
for v in "plain_w30:--warmup 30" "crc_w30:--inline-crc32 --warmup 30" "crc_w5:--inline-crc32 --warmup 5"; do
  name=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python3 bench.py $B $a > $O/bench_$name.json 2>/dev/null
  python3 -c "import json;d=json.load(open('$O/bench_$name.json'));print('$name', d['kernels']['encode']['ms'], d['kernels']['decode']['ms'], d['value']); print(d['step_ms'])"
done
