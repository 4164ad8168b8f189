# XCD-aware order for launches of >= 12 products only: config 4 and config 3 timing
rm -f gpurun_out/abm.txt
bash tools/ab_multi.sh "--model gru" X=0 AAC_GEMM_XCD_ALL=2 || exit 1
bash tools/ab_multi.sh "" X=0 AAC_GEMM_XCD_ALL=2
