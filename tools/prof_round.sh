export TMPDIR=/tmp
T="rocprofv3 --kernel-trace --output-format csv"
SHORT="--steps 10 --warmup 3 --no-cpu-baseline --env-micro 0"
bash tools/gpu_job.sh \
    "prof3:::240:::$T --stats -d gpurun_out/prof3 -o run -- python3 bench.py $SHORT" \
    "prof4:::240:::$T --stats -d gpurun_out/prof4 -o run -- python3 bench.py --model gru $SHORT" \
    "prof5:::240:::$T --stats -d gpurun_out/prof5 -o run -- python3 bench.py --model uam $SHORT"
