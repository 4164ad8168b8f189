export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "tests:::600:::python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_uam_learner_gpu.py tests/test_parallel_gpu.py tests/test_config_size_gpu.py -k 'uam or head or two_ranks'" \
  "b5:::200:::python bench.py --model uam --no-cpu-baseline --steps 50 --env-micro 0" \
  "b5b:::200:::python bench.py --model uam --no-cpu-baseline --steps 50 --env-micro 0"
for kv in AAC_NONE=1 AAC_ATTN_WGS=2048 AAC_ATTN_WGS=640 AAC_NONE=2; do
  env $kv timeout -k 10 120 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --env-micro 0 > gpurun_out/ab.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab.json') if l.startswith('{')][-1]); print('att $kv', round(d['ms_per_step'],4))" | tee -a gpurun_out/ab.txt
done
