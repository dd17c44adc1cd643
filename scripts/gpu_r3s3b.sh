# round-end rehearsal: full GPU test suite and the build entry's smoke() on the final tree
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_s3b.log 2>&1 \
  || { tail -30 gpurun_out/pytest_s3b.log; exit 1; }
tail -1 gpurun_out/pytest_s3b.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_s3b.log 2>&1 \
  || { tail -20 gpurun_out/smoke_s3b.log; exit 1; }
tail -2 gpurun_out/smoke_s3b.log
