SHORT="--no-cpu-baseline --env-micro 0"
bash tools/gpu_job.sh \
  "tail_tests:::400:::python -u -m pytest tests/test_step_tail_gpu.py tests/test_env_gpu.py tests/test_wgru_gpu.py tests/test_multimap_gpu.py -x -q --timeout 120 --timeout-method thread" \
  "b3:::150:::python bench.py $SHORT" \
  "b3_sep:::150:::AAC_FUSED_TAIL=0 python bench.py $SHORT" \
  "b4:::150:::python bench.py --model gru $SHORT" \
  "b4_sep:::150:::AAC_FUSED_TAIL=0 python bench.py --model gru $SHORT"
