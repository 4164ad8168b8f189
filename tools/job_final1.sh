# config-4 XCD A/B, then the round's bench evidence (three bench lines + kernel traces)
rm -f gpurun_out/abm.txt gpurun_out/job.log
bash tools/ab_multi.sh "--model gru" X=0 AAC_GEMM_XCD_ALL=2 || exit 1
bash tools/evidence_round.sh bench
