#!/bin/bash
# full GPU test tier, agent-loop bench, then a rocprofv3 kernel profile of the default bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/bench_agent.py ${AGENT_ARGS} --out gpurun_out/bench_agent.json > gpurun_out/bench_agent.log 2>&1; rc=$?
echo "agent bench rc=$rc"; tail -3 gpurun_out/bench_agent.log
[ $rc -eq 0 ] || exit $rc
TAG=default BENCH_ARGS="--steps 2 --warmup 1 --no-ingest" PROF_TIMEOUT=500 bash scripts/profile_bench.sh
