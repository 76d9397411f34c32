set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03ac; mkdir -p $O
timeout -k 10 400 python3 bench.py --gpus 2 --same-device --steps 20 --warmup 5 --no-host > $O/bench_2rank_same_device.json 2> $O/bench_2rank.err; tail -c 1500 $O/bench_2rank_same_device.json
