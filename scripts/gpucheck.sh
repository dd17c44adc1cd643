set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/smoke_final.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/bench_final.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_final.log; tail -2 gpurun_out/smoke_final.log; grep '^{' gpurun_out/bench_final.log | cut -c1-400; exit $rc
