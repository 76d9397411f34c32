set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03p; mkdir -p $O
export TMPDIR=/tmp
MB_RANDOM=1 timeout -k 10 200 tools/membench 10 ceil > $O/membench_ceil.txt 2>&1; grep "bpc=2" $O/membench_ceil.txt
timeout -k 10 300 python3 tools/ab_bench.py base ECAMD_ENC_NOCOMP=1 ECAMD_ENC_NOCOMP=1,ECAMD_EDGE_SIDE=2 ECAMD_ENC_NOCOMP=1,ECAMD_EDGE_BLOCKS=0 > $O/ab_b2b.txt 2>&1; cat $O/ab_b2b.txt
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/ab_bench.py --rounds 2 ECAMD_ENC_NOCOMP=1,ECAMD_EDGE_SIDE=2 > $GRAFT_REPO_ROOT/$O/prof.txt 2>&1)
python3 tools/rocpd_stats.py $O/prof > $O/kernel_stats.txt; head -6 $O/kernel_stats.txt
