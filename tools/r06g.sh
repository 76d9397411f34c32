set -e
O=gpurun_out/r06g; mkdir -p $O
ECAMD_REGISTER_CALLER=1 timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_inplace.log 2>&1
tail -2 $O/pytest_gpu_inplace.log
ECAMD_REGISTER_CALLER=1 timeout -k 10 300 python3 tools/swift_calls.py --procs 1,4,15 --seconds 1 > $O/swift_inplace.txt 2>&1
cat $O/swift_inplace.txt
timeout -k 10 300 python3 tools/swift_calls.py --procs 1,4,15 --seconds 1 > $O/swift_staged.txt 2>&1
cat $O/swift_staged.txt
