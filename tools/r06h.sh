set -e
O=gpurun_out/r06h; mkdir -p $O
export TMPDIR=/tmp
MB_RANDOM=1 timeout -k 10 240 tools/membench 20 "dmapat" > $O/membench.txt 2>&1
echo membench done
timeout -k 10 400 python3 tools/ab_bench.py --alt --rounds 5 base ECAMD_ENC_DMA=3,ECAMD_ENC_DMA_W=16 > $O/ab_enc_w16.txt 2>&1
cat $O/ab_enc_w16.txt | tail -6
timeout -k 10 400 python3 tools/ab_bench.py --full-stripe --rounds 5 base ECAMD_ENC_DATA_W=16 ECAMD_ENC_DATA_R=4 ECAMD_ENC_DATA_W=8,ECAMD_ENC_DATA_R=4 ECAMD_ENC_DATA_W=8 > $O/ab_full.txt 2>&1
cat $O/ab_full.txt | tail -8
timeout -k 10 400 python3 tools/ab_bench.py --m 2 --rounds 5 base ECAMD_ENC_DMA2=1 > $O/ab_m2.txt 2>&1
cat $O/ab_m2.txt | tail -6
for f in pmc1 pmc2 pmc4; do
  (cd /tmp && timeout -s KILL 150 rocprofv3 -i $GRAFT_REPO_ROOT/tools/$f.txt --output-format csv -d $GRAFT_REPO_ROOT/$O/sq_$f -o run -- python3 $GRAFT_REPO_ROOT/tools/ab_bench.py --m 2 --rounds 1 --settle-ms 20 base ECAMD_ENC_DMA2=1 > $GRAFT_REPO_ROOT/$O/sq_$f.log 2>&1)
done
python3 tools/pmc_table.py $O/sq_pmc1 $O/sq_pmc2 $O/sq_pmc4 > $O/sq_table_m2.txt 2>&1 || true
cat $O/sq_table_m2.txt | head -60
