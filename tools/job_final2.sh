# round-end evidence: full GPU test suite, the three bench lines + kernel traces, the PMC passes
mkdir -p gpurun_out
rm -f gpurun_out/job.log
timeout -k 10 560 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.txt
[ $rc -le 1 ] || exit $rc
bash tools/evidence_round.sh bench > /dev/null || exit 1
bash tools/evidence_round.sh pmc > /dev/null
tail -3 gpurun_out/job.log
