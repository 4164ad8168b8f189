# GRU learner GEMM traffic: FETCH/WRITE passes for the default tile policy and an alternative knob
export TMPDIR=/tmp
T="rocprofv3 --kernel-trace --output-format csv"
SHORT="--model gru --steps 10 --warmup 3 --no-cpu-baseline --env-micro 0"
KV="${1:-AAC_GEMM_XCD_ALL=1}"
bash tools/gpu_job.sh \
  "f0:::90:::timeout -s KILL 80 $T --pmc FETCH_SIZE -d gpurun_out/pg_f0 -o run -- python3 bench.py $SHORT" \
  "w0:::90:::timeout -s KILL 80 $T --pmc WRITE_SIZE -d gpurun_out/pg_w0 -o run -- python3 bench.py $SHORT" \
  "f1:::90:::$KV AAC_GEMM_DUMP=60 timeout -s KILL 80 $T --pmc FETCH_SIZE -d gpurun_out/pg_f1 -o run -- python3 bench.py $SHORT" \
  "w1:::90:::$KV timeout -s KILL 80 $T --pmc WRITE_SIZE -d gpurun_out/pg_w1 -o run -- python3 bench.py $SHORT"
bash tools/ab_multi.sh "--model gru" X=0 "$KV"
