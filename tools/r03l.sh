set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03l; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; tail -2 $O/pytest_gpu.log
timeout -k 10 300 python3 tools/ab_bench.py --alt --crc base ECAMD_CRC_RUN=0 ECAMD_CRC_RUN=4 ECAMD_CRC_RUN=16 > $O/ab_crc.txt 2>&1; cat $O/ab_crc.txt
timeout -k 10 300 python3 bench.py --inline-crc32 --steps 10 --no-host --no-cpu-baseline > $O/bench_crc.json 2>/dev/null; python3 -c "import json;d=json.load(open('$O/bench_crc.json'));print('crc run8', d['kernels'])"
ECAMD_CRC_RUN=0 timeout -k 10 300 python3 bench.py --inline-crc32 --steps 10 --no-host --no-cpu-baseline > $O/bench_crc_run0.json 2>/dev/null; python3 -c "import json;d=json.load(open('$O/bench_crc_run0.json'));print('crc run0', d['kernels'])"
MB_RANDOM=1 timeout -k 10 200 tools/membench 10 ceil > $O/membench_ceil.txt 2>&1; cat $O/membench_ceil.txt
timeout -k 10 300 python3 tools/ab_bench.py --alt base ECAMD_ENC_NOCOMP=1 ECAMD_ENC_NTL=1 > $O/ab_alt.txt 2>&1; cat $O/ab_alt.txt
timeout -k 10 300 python3 tools/ab_bench.py base ECAMD_ENC_NOCOMP=1 ECAMD_ENC_NTL=1 > $O/ab_b2b.txt 2>&1; cat $O/ab_b2b.txt
timeout -k 10 300 python3 tools/ab_bench.py --full-stripe --alt base ECAMD_DATA_COPY=1 > $O/ab_full.txt 2>&1; cat $O/ab_full.txt
timeout -k 10 200 python3 tools/fresh_probe.py > $O/fresh_probe.txt 2>&1; cat $O/fresh_probe.txt
