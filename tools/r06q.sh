set -e
O=gpurun_out/r06q; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_dma.py tests/test_gpu_decode_variants.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
timeout -k 10 500 python3 tools/ab_bench.py --alt --rounds 5 base ECAMD_DEC_ALIGN=0 ECAMD_DEC_DMA=4,ECAMD_DEC_DMA_L=4,ECAMD_DEC_DMA_W=8 ECAMD_DEC_DMA=4,ECAMD_DEC_DMA_L=2,ECAMD_DEC_DMA_W=8 ECAMD_DEC_DMA=3,ECAMD_DEC_DMA_L=4,ECAMD_DEC_DMA_W=16 > $O/ab_align.txt 2>&1
tail -7 $O/ab_align.txt
