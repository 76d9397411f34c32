set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03v; mkdir -p $O
MB_RANDOM=1 timeout -k 10 200 tools/membench 10 wpb > $O/membench_wpb.txt 2>&1; cat $O/membench_wpb.txt
MB_RANDOM=1 timeout -k 10 200 tools/membench 10 wpb > $O/membench_wpb2.txt 2>&1; cat $O/membench_wpb2.txt
(timeout -k 10 400 python3 tools/swift_mix.py > $O/swift_mix.json 2> $O/swift_mix.err); head -c 600 $O/swift_mix.json
