set -e
O=gpurun_out/r06ak; mkdir -p $O
export TMPDIR=/tmp
for f in pmc1 pmc2 pmc9; do
  (cd /tmp && timeout -s KILL 150 rocprofv3 -i $GRAFT_REPO_ROOT/tools/$f.txt --output-format csv -d $GRAFT_REPO_ROOT/$O/sq_$f -o run -- python3 $GRAFT_REPO_ROOT/tools/ab_bench.py --crc --rounds 1 --settle-ms 20 base ECAMD_CRC_V=10 > $GRAFT_REPO_ROOT/$O/sq_$f.log 2>&1)
done
python3 tools/pmc_table.py $O/sq_pmc1 $O/sq_pmc2 $O/sq_pmc9 > $O/sq_table_crc.txt 2>&1 || true
grep -A20 "encode_dma_kernel" $O/sq_table_crc.txt | grep -E "encode_dma|VALU|LDS|MFMA|BUSY_CYCLES|GRBM" | head -40
