# GPU: numerics of the deferred split-K norm, then bench A/B (reduce folded into RMSNorm vs separate)
# and the in-flight sweep.  Usage: bash scripts/ab_defer.sh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "splitk or rmsnorm" > gpurun_out/t_defer.log 2>&1 || { tail -30 gpurun_out/t_defer.log; exit 1; }
tail -2 gpurun_out/t_defer.log
run() {  # tag env-assignments... -- bench args
  local tag=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/ab_$tag.log 2>&1 || return $?
  grep '^{' gpurun_out/ab_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['engine_per_timed_step']; print('$tag', d['value'], d['p50_ttft_ms'], d['ms_per_step'], e['decode_s'], e['prefill_s'], e['decode_steps'])"
}
run defer0_if6 GRAG_DEFER_SPLITK=0 python -u bench.py --no-ingest --agent-jobs 0 --inflight 6 &&
run defer1_if6 GRAG_DEFER_SPLITK=1 python -u bench.py --no-ingest --agent-jobs 0 --inflight 6 &&
run defer1_if3 GRAG_DEFER_SPLITK=1 python -u bench.py --no-ingest --agent-jobs 0 --inflight 3 &&
run defer1_if8 GRAG_DEFER_SPLITK=1 python -u bench.py --no-ingest --agent-jobs 0 --inflight 8 &&
run defer1_if7 GRAG_DEFER_SPLITK=1 python -u bench.py --no-ingest --agent-jobs 0 --inflight 7
