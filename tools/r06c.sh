set -e
O=gpurun_out/r06c; mkdir -p $O
export MB_RANDOM=1
timeout -k 10 240 tools/membench 20 "roof dmapat" > $O/membench.txt 2>&1
echo membench done
PYECLIB_AMD_LIBRARY=$PWD/tools/build/libpyeclib_amd_checks.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_edges.py tests/test_gpu_decode_variants.py tests/test_gpu_multiproc.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_checked.log 2>&1
tail -2 $O/pytest_checked.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host --swift-procs "" --fresh-steps 0 > $O/bench.json 2> $O/bench.err
echo bench done
