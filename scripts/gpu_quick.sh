# Quick GPU pass: the given pytest selection (default: all GPU tests), then the default bench.
set -o pipefail
mkdir -p gpurun_out
SEL=${1:-tests}
TAG=${2:-quick}
timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 800 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.log 2>&1
rc=$?
grep '^{' gpurun_out/bench_$TAG.log | cut -c1-400
grep "agent e2e\|ingest:\|serving:" gpurun_out/bench_$TAG.log
exit $rc
