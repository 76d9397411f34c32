set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03f; mkdir -p $O
V="base ECAMD_ENC_NOCOMP=1,ECAMD_ENC_PER_CU=2 ECAMD_ENC_NOCOMP=1,ECAMD_ENC_PER_CU=2,ECAMD_EDGE_SIDE=1 ECAMD_ENC_NOCOMP=1,ECAMD_ENC_PER_CU=2,ECAMD_EDGE_SIDE=2 ECAMD_ENC_PER_CU=2,ECAMD_EDGE_SIDE=2 ECAMD_ENC_PER_CU=2 ECAMD_ENC_NTL=1,ECAMD_ENC_PER_CU=2"
timeout -k 10 300 python3 tools/ab_bench.py $V > $O/ab_b2b.txt 2>&1; cat $O/ab_b2b.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/ab_bench.py --rounds 2 ECAMD_ENC_PER_CU=2,ECAMD_EDGE_SIDE=2 > $GRAFT_REPO_ROOT/$O/prof.txt 2>&1
find $GRAFT_REPO_ROOT/$O/prof -name '*kernel_stats.csv' -exec cp {} $GRAFT_REPO_ROOT/$O/kernel_stats.csv \;
cut -c1-200 $GRAFT_REPO_ROOT/$O/kernel_stats.csv
