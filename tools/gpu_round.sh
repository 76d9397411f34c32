#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, kernel-trace stats and the
# two HBM PMC passes (FETCH_SIZE / WRITE_SIZE in separate runs).  Every GPU
# step has its own time limit and the first failure ends the script.
#   tools/gpu_round.sh TAG [tests|smoke|ab|bench|prof|pmc ...]   (default: all but ab)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r01}
shift || true
STEPS=${*:-tests smoke bench prof pmc}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for s in $STEPS; do
  echo "== $s $(date +%T)"
  case $s in
  tests)
    (cd $R && timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 \
        --timeout-method thread > $O/pytest_gpu.log 2>&1)
    tail -3 $O/pytest_gpu.log ;;
  tracetests)
    # the whole GPU suite once under a kernel + memory-copy trace, so that a
    # fault names the last dispatch or copy before it
    (cd $R && timeout -k 10 900 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
        -d $O/trace -o run -- python3 -u -m pytest tests -m gpu -x -v --timeout 300 \
        --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1)
    tail -3 $O/pytest_gpu.log ;;
  newtests)
    (cd $R && timeout -k 10 600 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 300 \
        --timeout-method thread > $O/pytest_gpu_new.log 2>&1)
    tail -3 $O/pytest_gpu_new.log ;;
  membench)
    (cd $R && timeout -k 10 300 tools/membench ${MB_REPS:-20} ${MB_SECTIONS:-} > $O/membench.txt 2>&1)
    cat $O/membench.txt ;;
  multirank)
    (cd $R && timeout -k 10 600 python3 -u -m pytest tests/test_gpu_multirank.py -m gpu -x -v --timeout 300 \
        --timeout-method thread > $O/pytest_multirank.log 2>&1)
    tail -3 $O/pytest_multirank.log ;;
  config0)
    (cd $R && timeout -k 10 400 python3 bench.py --no-host --no-cpu-baseline --config0 --steps 5 \
        > $O/config0_bench.json 2> $O/config0_bench.err)
    tail -c 900 $O/config0_bench.json ;;
  sysfs)
    (ls /sys/class/kfd/kfd/topology/nodes/; for n in /sys/class/kfd/kfd/topology/nodes/*; do \
      echo "== $n"; grep -E "simd_count|location_id|domain|drm_render_minor" $n/properties; done; \
      echo "== numa"; for d in /sys/class/drm/card*/device; do echo "$d $(cat $d/numa_node 2>/dev/null)"; done; \
      cat /sys/devices/system/node/node*/cpulist; nproc; python3 -c "import os; print(len(os.sched_getaffinity(0)))"; \
      echo "ROCR=$ROCR_VISIBLE_DEVICES HIP=$HIP_VISIBLE_DEVICES CUDA=$CUDA_VISIBLE_DEVICES") > $O/sysfs.txt 2>&1 || true
    cat $O/sysfs.txt ;;
  smoke)
    (cd $R && timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1)
    tail -1 $O/smoke.log ;;
  ab)
    (cd $R && timeout -k 10 400 python3 tools/ab_bench.py ${AB:-base ECAMD_DEC_OCC3=1 ECAMD_XCD=0} > $O/ab.txt 2>&1)
    cat $O/ab.txt ;;
  abalt)
    (cd $R && timeout -k 10 400 python3 tools/ab_bench.py --alt ${AB:-base} > $O/ab_alt.txt 2>&1)
    cat $O/ab_alt.txt ;;
  abfull)
    (cd $R && timeout -k 10 400 python3 tools/ab_bench.py --full-stripe ${ABF:-base ECAMD_DATA_COPY=1} > $O/ab_full.txt 2>&1)
    cat $O/ab_full.txt ;;
  single)
    (cd $R && timeout -k 10 300 python3 tools/single_ab.py > $O/single_ab.txt 2>&1)
    cat $O/single_ab.txt ;;
  timeline)
    python3 $R/tools/rocpd_timeline.py $O/prof --last 24 > $O/timeline.txt 2>&1 || true
    cat $O/timeline.txt ;;
  config3)
    (cd $R && timeout -k 10 400 python3 bench.py --ec-type isa_l_rs_cauchy --k 12 --m 4 \
        --obj-bytes 16777216 --batch 128 --second reconstruct --steps 10 --no-host \
        > $O/config3_bench.json 2> $O/config3_bench.err)
    tail -c 700 $O/config3_bench.json ;;
  swift)
    (cd $R && timeout -k 10 400 python3 tools/swift_mix.py > $O/swift_mix.json 2> $O/swift_mix.err)
    head -c 400 $O/swift_mix.json ;;
  crc)
    (cd $R && timeout -k 10 300 python3 bench.py --inline-crc32 --steps 20 --warmup 5 --no-host \
        --no-cpu-baseline > $O/bench_crc.json 2> $O/bench_crc.err)
    tail -c 400 $O/bench_crc.json ;;
  bench)
    (cd $R && timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err)
    cat $O/bench.json ;;
  prof)
    # per-dispatch kernel trace of the bench's headline steps (no extra legs,
    # so the last 20 dispatches of each kernel are the timed steps), summarised
    # into kernel_stats.json for bench.py's roofline (frac_rocprof)
    (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
      -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-verify --no-host --crc-steps 0 \
      --fresh-steps 0 --full-stripe-steps 0 > $O/prof_bench.json 2> $O/prof.err)
    cat $O/prof_bench.json
    python3 $R/tools/kernel_stats_summary.py $O/prof $O/kernel_stats.json --steps 20
    find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \; ;;
  pmc)
    (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run \
      -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-verify --no-host --crc-steps 0 > $O/pmc_fetch.log 2>&1)
    (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run \
      -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-verify --no-host --crc-steps 0 > $O/pmc_write.log 2>&1)
    python3 $R/tools/pmc_summary.py $O/pmc_fetch $O/pmc_write $O/pmc_summary.json ;;
  list)
    (cd /tmp && timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1) || true
    grep -c . $O/counters.txt ;;
  sq)
    for f in ${SQ_FILES:-pmc1 pmc2 pmc3}; do
      (cd /tmp && timeout -s KILL 150 rocprofv3 -i $R/tools/$f.txt --output-format csv -d $O/sq_$f -o run \
        -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-verify --no-host --crc-steps 0 ${SQ_ARGS:-} > $O/sq_$f.log 2>&1)
    done
    python3 $R/tools/pmc_table.py $(for f in ${SQ_FILES:-pmc1 pmc2 pmc3}; do echo $O/sq_$f; done) > $O/sq_table.txt 2>&1 || true
    cat $O/sq_table.txt ;;
  *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "gpu_round $TAG done: $STEPS"
