# config-4 env options, interleaved: default (separate push / reset), fused tail, fused tail with
# 32-agent workgroups (4 envs: one round of 1024 workgroups), 32-agent workgroups alone
mkdir -p gpurun_out
for i in 1 2; do
  for kv in "X=0" "AAC_FUSED_TAIL=1" "AAC_FUSED_TAIL=1 AAC_ENV_AGENTS_PER_WG=32" "AAC_ENV_AGENTS_PER_WG=32"; do
    timeout -k 10 150 env $kv python bench.py --model gru --no-cpu-baseline --env-micro 0 --steps 60 > gpurun_out/abg.log 2>&1 || exit 1
    python -c "import json; d=[json.loads(l) for l in open('gpurun_out/abg.log') if l.startswith('{')][-1]; print('$kv', round(d['ms_per_step'],4), round(d['env_roofline']['avg_launch_ms'],4))" | tee -a gpurun_out/abg.txt
  done
done
