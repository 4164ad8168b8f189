#!/bin/bash
# Round-4 PMC evidence at config 3 (bench.py defaults, short run) on the GPU box (repo root):
#   FETCH_SIZE / WRITE_SIZE passes (HBM bytes of every kernel: the attention kernels, the grouped GEMM
#   -> profiles/gemm_pmc.json and the env step tail -> profiles/env_step_pmc.json, which bench.py
#   reads), an SQ pass for the attention kernels
#   (instruction mix, MFMA busy, waits) and an fp64 SQ pass for the env step kernel; each --pmc pass
#   is its own run with no trace domains, under its own time limit (tools/gpu_job.sh stops at the
#   first crash or timeout).  Summaries go to gpurun_out/ and profiles/ (the box's copy: a bench run
#   later in the same call reads them).
export TMPDIR=/tmp
T="rocprofv3 --kernel-trace --output-format csv"
SHORT="--steps 10 --warmup 3 --no-cpu-baseline --env-micro 0"
SQA="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS"
SQF="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY"
bash tools/gpu_job.sh \
  "pf:::90:::timeout -s KILL 80 $T --pmc FETCH_SIZE -d gpurun_out/p4f -o run -- python3 bench.py $SHORT" \
  "pw:::90:::timeout -s KILL 80 $T --pmc WRITE_SIZE -d gpurun_out/p4w -o run -- python3 bench.py $SHORT" \
  "pa:::90:::timeout -s KILL 80 $T --pmc $SQA -d gpurun_out/p4a -o run -- python3 bench.py $SHORT" \
  "pd:::90:::timeout -s KILL 80 $T --pmc $SQF -d gpurun_out/p4d -o run -- python3 bench.py $SHORT" \
  "sum:::60:::python3 tools/pmc_kernels.py gpurun_out/r04_attn_pmc.json --fetch gpurun_out/p4f/run_counter_collection.csv --write gpurun_out/p4w/run_counter_collection.csv --sq gpurun_out/p4a/run_counter_collection.csv --kernel attn_enc_kernel=attn_enc_kernel --kernel attn_mfma_bwd_kernel=attn_mfma_bwd_kernel --kernel gemm_kernel=gemm_kernel envs=4096 agents=5 batch=1024 && python3 tools/pmc_kernels.py gpurun_out/env_fp64_pmc.json --fetch gpurun_out/p4f/run_counter_collection.csv --write gpurun_out/p4w/run_counter_collection.csv --sq gpurun_out/p4d/run_counter_collection.csv --kernel 'step_kernel=step_kernel<0, 2, true>' envs=4096 agents=5 radar=combined && python3 tools/pmc_summary.py gpurun_out/p4f/run_counter_collection.csv gpurun_out/p4w/run_counter_collection.csv gemm_kernel mean gpurun_out/gemm_pmc.json model=att envs=4096 agents=5 batch=1024 algorithmic_bytes_per_launch=22510019 && python3 tools/pmc_summary.py gpurun_out/p4f/run_counter_collection.csv gpurun_out/p4w/run_counter_collection.csv 'step_kernel<0, 2, true>' median gpurun_out/env_step_pmc.json envs=4096 agents=5 radar=combined variant=att maps=1 tail=1 algorithmic_bytes_per_launch=24125440 && cp gpurun_out/r04_attn_pmc.json gpurun_out/env_fp64_pmc.json gpurun_out/gemm_pmc.json gpurun_out/env_step_pmc.json profiles/"
