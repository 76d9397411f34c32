set -e
O=gpurun_out/r06k; mkdir -p $O
MB_RANDOM=1 timeout -k 10 240 tools/membench 20 "dmapat" > $O/membench.txt 2>&1
grep -E "dma enc W12 R3" $O/membench.txt
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host --swift-procs "" --fresh-steps 0 > $O/bench.json 2> $O/bench.err
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac_by_kernel'], d.get('encode_full_stripe'))"
