set -e
O=gpurun_out/r06al; mkdir -p $O
export TMPDIR=/tmp
for km in "10 2" "12 2"; do set -- $km
  for f in pmc1 pmc2; do
    (cd /tmp && timeout -s KILL 150 rocprofv3 -i $GRAFT_REPO_ROOT/tools/$f.txt --output-format csv -d $GRAFT_REPO_ROOT/$O/k$1_$f -o run -- python3 $GRAFT_REPO_ROOT/tools/ab_bench.py --k $1 --m $2 --rounds 1 --settle-ms 20 base > $GRAFT_REPO_ROOT/$O/k$1_$f.log 2>&1)
  done
  python3 tools/pmc_table.py $O/k$1_pmc1 $O/k$1_pmc2 > $O/sq_k$1_m$2.txt 2>&1 || true
  echo "k=$1 m=$2"; grep -A18 "encode_dma_kernel" $O/sq_k$1_m$2.txt | grep -E "encode_dma|INSTS_VALU|INSTS_LDS|LDS_IDX|BANK|BUSY_CYCLES|GRBM|VMEM|WAIT_INST_ANY|WAVE_CYCLES"
done
