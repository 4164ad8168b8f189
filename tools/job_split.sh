# new split-K / LDS-tile defaults: learner parity tests, then the three benches
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_gpu.py tests/test_config_size_gpu.py \
  tests/test_learner_gpu.py tests/test_parallel_gpu.py tests/test_gru_gpu.py tests/test_step_tail_gpu.py > gpurun_out/sp_tests.log 2>&1 || { tail -30 gpurun_out/sp_tests.log; exit 1; }
tail -2 gpurun_out/sp_tests.log
rm -f gpurun_out/abm.txt
bash tools/ab_multi.sh "--model gru" X=0 || exit 1
bash tools/ab_multi.sh "--model uam" X=0
