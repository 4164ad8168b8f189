# A/B of one env knob on the config-3 bench, interleaved (A B A B A B) to average out run-to-run drift:
#   bash tools/ab_knob.sh "AAC_ATTN_WN=0" "AAC_ATTN_WN=1" [extra bench args]
A="$1"; B="$2"; shift 2
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in A B; do
    kv=$([ $v = A ] && echo "$A" || echo "$B")
    timeout -k 10 150 env $kv python bench.py --no-cpu-baseline --env-micro 0 --steps 100 "$@" > gpurun_out/ab_$v$i.log 2>&1 || exit 1
    python -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/ab_$v$i.log') if l.startswith('{')][-1]; print('$v', '$kv', round(d['ms_per_step'],4))" | tee -a gpurun_out/ab.txt
  done
done
