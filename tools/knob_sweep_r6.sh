# GEMM tile-policy knobs on the config-3 schedule: bash tools/knob_sweep_r6.sh (GPU box)
for i in 1 2; do
for kv in "NONE=0" "AAC_GEMM_LDS_SMALL=1" "AAC_GEMM_LDS_PREF_WG=768" "AAC_GEMM_LDS_PREF_WG=384" "AAC_GEMM_LDS_MIN_K=32" "AAC_GEMM_DEEP_CHAIN=1" "AAC_GEMM_XCD=1"; do
  env $kv python bench.py --no-cpu-baseline --env-micro 0 --no-seg-overhead > gpurun_out/s.log 2>&1 || exit 3
  echo "$kv $(grep '^{' gpurun_out/s.log | cut -c1-200)"
done; done
