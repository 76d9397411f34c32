set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03y; mkdir -p $O
MB_RANDOM=1 timeout -k 10 200 tools/membench 10 wpb > $O/membench_wpb.txt 2>&1; cat $O/membench_wpb.txt
