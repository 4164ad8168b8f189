cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS -d $R/gpurun_out/pmc/a -o run --output-format csv -- python3 $R/tools/mb_lds.py 0 && \
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc/b -o run --output-format csv -- python3 $R/tools/mb_lds.py 0 && \
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/pmc/c -o run --output-format csv -- python3 $R/tools/mb_lds.py 0 && \
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/gpurun_out/pmc/d -o run --output-format csv -- python3 $R/tools/mb_lds.py 0
