# float64 learner knobs on the config-5 schedule: bash tools/knob_sweep_r6_uam.sh (GPU box)
for i in 1 2; do
for kv in "NONE=0" "AAC_UAM_KS=2" "AAC_UAM_KS=8" "AAC_GEMM64_KW4=0" "AAC_GEMM64_KW4_STEPS=8" "AAC_GEMM64_KW4_STEPS=32" "AAC_GEMM64_KW4_TILES=256"; do
  env $kv python bench.py --model uam --no-cpu-baseline --env-micro 0 --no-seg-overhead > gpurun_out/s.log 2>&1 || exit 3
  echo "$kv $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s.log)"
done; done
