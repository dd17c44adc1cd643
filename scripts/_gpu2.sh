#!/bin/bash
# GPT-2 GPU tests + agent-loop bench (BASELINE config 5) on one GPU
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpt2.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpt2.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpt2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/bench_agent.py ${AGENT_ARGS} --out gpurun_out/bench_agent.json > gpurun_out/bench_agent.log 2>&1; rc=$?
echo "agent bench rc=$rc"; tail -6 gpurun_out/bench_agent.log
exit $rc
