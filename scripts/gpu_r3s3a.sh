# engine GPU tests + default bench after the decode post fast path change
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_s3d.log 2>&1 \
  || { tail -30 gpurun_out/pytest_s3d.log; exit 1; }
tail -1 gpurun_out/pytest_s3d.log
timeout -k 10 700 python -u bench.py > gpurun_out/bench_s3d.log 2>&1 || { tail -20 gpurun_out/bench_s3d.log; exit 1; }
grep '^{' gpurun_out/bench_s3d.log | cut -c1-220
grep "serving:\|agent e2e\|ingest:" gpurun_out/bench_s3d.log
