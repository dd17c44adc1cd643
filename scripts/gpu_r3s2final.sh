# end-of-session pass: full GPU test suite, default bench, rocprofv3 kernel summary of the serving phase
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_final.log 2>&1 \
  || { tail -30 gpurun_out/pytest_final.log; exit 1; }
tail -1 gpurun_out/pytest_final.log
timeout -k 10 700 python -u bench.py > gpurun_out/bench_final.log 2>&1 || { tail -20 gpurun_out/bench_final.log; exit 1; }
grep '^{' gpurun_out/bench_final.log | cut -c1-200
grep "serving:\|agent e2e\|ingest:" gpurun_out/bench_final.log
bash scripts/profile_bench.sh > gpurun_out/prof_summary_final.txt 2>&1 || { tail -20 gpurun_out/prof_summary_final.txt; exit 1; }
head -14 gpurun_out/prof_summary_final.txt
