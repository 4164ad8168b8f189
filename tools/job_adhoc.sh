export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "all:::900:::python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/" \
  "smoke:::200:::python -c 'import __graft_entry__ as g; g.smoke()'" && bash tools/evidence_round.sh bench
