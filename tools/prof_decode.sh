#!/bin/bash
# PMC passes of a short bench run, for the current decode path and (with
# ECAMD_DPLAIN=1) the plain-copy path.  Output: gpurun_out/pmc/<mode>/<pass>.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
i=0
for mode in shift plain; do
  if [ $mode = shift ]; then export ECAMD_DSHIFT=1; else unset ECAMD_DSHIFT; fi
  for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
             "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --pmc $ctr --output-format csv -d $R/gpurun_out/pmc/$mode/p$i -o run \
      -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc/$mode.p$i.log 2>&1
  done
done
python3 $R/tools/pmc_table.py $R/gpurun_out/pmc/shift > $R/gpurun_out/pmc/shift.txt
python3 $R/tools/pmc_table.py $R/gpurun_out/pmc/plain > $R/gpurun_out/pmc/plain.txt
