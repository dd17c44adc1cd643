# GPU: bench queries/s and p50 TTFT by in-flight batches (serving phase only).
# Usage: bash scripts/sweep_inflight.sh "3 6 8" [steps]
set -o pipefail
mkdir -p gpurun_out
for f in ${1:-3 6 8}; do
  timeout -k 10 300 python -u bench.py --no-ingest --agent-jobs 0 --inflight $f --steps ${2:-3} > gpurun_out/inflight_$f.log 2>&1 || exit $?
  grep '^{' gpurun_out/inflight_$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['engine_per_timed_step']; print($f, d['value'], d['p50_ttft_ms'], d['ms_per_step'], e['decode_s'], e['prefill_s'], e['decode_steps'], d['steady_state_decode_ratio'])"
done
