set -euo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03ag; mkdir -p $O
timeout -k 10 200 python3 tools/fresh_probe.py > $O/fresh_probe.txt 2>&1; cat $O/fresh_probe.txt
bash tools/gpu_round.sh r03ag tests smoke bench pmc
