# env workgroup sizing + config-4 fused tail: env / tail / GRU parity, then configs 3 and 4 benches
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_step_tail_gpu.py tests/test_env_gpu.py tests/test_wgru_gpu.py tests/test_gru_gpu.py > gpurun_out/epb_tests.log 2>&1 || { tail -30 gpurun_out/epb_tests.log; exit 1; }
tail -3 gpurun_out/epb_tests.log
timeout -k 10 200 python bench.py --model gru --no-cpu-baseline --steps 100 > gpurun_out/epb_b4.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/epb_b3.log 2>&1 || exit 1
python - <<'P'
import json
for f in ("gpurun_out/epb_b4.log", "gpurun_out/epb_b3.log"):
    d = [json.loads(l) for l in open(f) if l.startswith("{")][-1]
    print(f, d["value"], d["ms_per_step"], d["env_roofline"]["avg_launch_ms"], d["roofline"]["frac"])
P
