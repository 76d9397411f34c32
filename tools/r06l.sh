set -e
O=gpurun_out/r06l; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host --swift-procs "" --fresh-steps 0 > $O/bench.json 2> $O/bench.err
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac_by_kernel'], d.get('encode_full_stripe'))"
