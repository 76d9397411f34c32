set -e
O=gpurun_out/r06am; mkdir -p $O
export TMPDIR=/tmp
for km in "10 2" "12 2"; do set -- $km
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$O/k$1_fetch -o run -- python3 $GRAFT_REPO_ROOT/tools/ab_bench.py --k $1 --m $2 --rounds 1 --settle-ms 20 base > $GRAFT_REPO_ROOT/$O/k$1_fetch.log 2>&1)
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$O/k$1_write -o run -- python3 $GRAFT_REPO_ROOT/tools/ab_bench.py --k $1 --m $2 --rounds 1 --settle-ms 20 base > $GRAFT_REPO_ROOT/$O/k$1_write.log 2>&1)
  python3 tools/pmc_table.py $O/k$1_fetch $O/k$1_write > $O/traffic_k$1.txt 2>&1 || true
  echo "k=$1 m=$2"; grep -A3 "encode_dma_kernel<Gf16<1>, $1, 2, 3" $O/traffic_k$1.txt
done
