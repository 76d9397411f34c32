set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03j; mkdir -p $O
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --inline-crc32 --steps 10 --warmup 2 --no-cpu-baseline --no-verify --no-host > $GRAFT_REPO_ROOT/$O/bench_crc.json 2> $GRAFT_REPO_ROOT/$O/prof.err)
python3 tools/rocpd_stats.py $O/prof > $O/kernel_stats.txt; head -8 $O/kernel_stats.txt
python3 tools/rocpd_timeline.py $O/prof --last 30 > $O/timeline.txt 2>&1 || true; cat $O/timeline.txt
timeout -k 10 300 python3 tools/ab_bench.py --alt --crc base ECAMD_CRC_PER_CU=8 > $O/ab_crc.txt 2>&1; cat $O/ab_crc.txt
