set -e
O=gpurun_out/r06ag; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dma.py tests/test_gpu_api.py tests/test_gpu_configs.py tests/test_gpu_edges.py -m gpu -x -q -k "crc or reconstruct" --timeout 300 --timeout-method thread > $O/pytest_crc.log 2>&1
tail -2 $O/pytest_crc.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --inline-crc32 --steps 20 --warmup 5 --no-cpu-baseline --no-verify --no-host --fresh-steps 0 --full-stripe-steps 0 > $GRAFT_REPO_ROOT/$O/prof_bench.json 2> $GRAFT_REPO_ROOT/$O/prof.err
python3 -c "
import csv,glob
f=glob.glob('$GRAFT_REPO_ROOT/$O/prof/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)): print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1000,1), round(float(r['MinNs'])/1000,1))
"
