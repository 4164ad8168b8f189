export TMPDIR=/tmp
for m in gru att; do
for kv in AAC_NONE=1 AAC_GEMM_XCD_ALL=1 AAC_NONE=2 AAC_GEMM_XCD_ALL=2; do
  env $kv timeout -k 10 120 python bench.py --model $m --steps 40 --warmup 5 --no-cpu-baseline --env-micro 0 > gpurun_out/ab.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab.json') if l.startswith('{')][-1]); print('$m $kv', round(d['ms_per_step'],4), round(d['roofline']['frac'],4), round(d['roofline']['gemm_ms_per_update'],4))" | tee -a gpurun_out/ab.txt
done
done
