set -e
O=gpurun_out/r06i; mkdir -p $O
export TMPDIR=/tmp
MB_RANDOM=1 timeout -k 10 240 tools/membench 20 "dmapat" > $O/membench.txt 2>&1
echo membench done
timeout -k 10 500 python3 tools/ab_bench.py --alt --rounds 5 base ECAMD_ENC_DMA=4 ECAMD_ENC_DMA=5 ECAMD_DEC_DMA=4,ECAMD_DEC_DMA_L=2,ECAMD_DEC_DMA_W=8 ECAMD_DEC_DMA=5,ECAMD_DEC_DMA_L=2,ECAMD_DEC_DMA_W=8 > $O/ab_alt.txt 2>&1
tail -7 $O/ab_alt.txt
timeout -k 10 400 python3 tools/ab_bench.py --full-stripe --rounds 5 base ECAMD_ENC_DATA_W=8,ECAMD_ENC_DATA_R=5 ECAMD_ENC_DATA_W=12,ECAMD_ENC_DATA_R=3 > $O/ab_full.txt 2>&1
tail -5 $O/ab_full.txt
timeout -k 10 400 python3 tools/ab_bench.py --m 2 --rounds 5 base ECAMD_ENC_STREAM2=1 > $O/ab_m2.txt 2>&1
tail -4 $O/ab_m2.txt
