#!/bin/bash
# GPU validation: kernel/engine tests, then a short bench. Stops on crash/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -q --timeout 300 ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "$SKIP_BENCH" ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-900} python bench.py ${BENCH_ARGS:---steps 2 --warmup 1 --no-ingest} > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -25 gpurun_out/bench.log
exit $rc
