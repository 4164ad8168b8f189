# interleaved A/B/C... of env knobs on one bench config:  bash tools/ab_multi.sh "<bench args>" "K=V" "K=V K2=V2" ...
ARGS="$1"; shift
mkdir -p gpurun_out
for i in 1 2 3; do
  for kv in "$@"; do
    timeout -k 10 150 env $kv python bench.py --no-cpu-baseline --env-micro 0 --steps 100 $ARGS > gpurun_out/abm.log 2>&1 || exit 1
    python -c "import json; d=[json.loads(l) for l in open('gpurun_out/abm.log') if l.startswith('{')][-1]; print('$kv', round(d['ms_per_step'],4), round(d['roofline'].get('frac',0),4))" | tee -a gpurun_out/abm.txt
  done
done
