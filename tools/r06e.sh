set -e
O=gpurun_out/r06e; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_caller_buffers.py tests/test_gpu_api.py tests/test_gpu_multiproc.py tests/test_gpu_concurrency.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -3 $O/pytest.log
timeout -k 10 300 python3 tools/single_probe.py --sizes 65536,1048576,4194304 --reps 30 --direct 0,1 > $O/single_probe.txt 2>&1
cat $O/single_probe.txt
