# GPU: throughput / TTFT trade-off by arrival-group size at the default depth (serving phase only).
set -o pipefail
mkdir -p gpurun_out
for a in 4 16 8; do
  timeout -k 10 300 python -u bench.py --no-ingest --agent-jobs 0 --arrival-groups $a --steps 4 > gpurun_out/arrival_$a.log 2>&1 || exit $?
  grep '^{' gpurun_out/arrival_$a.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['engine_per_timed_step']; print('groups $a', d['value'], d['p50_ttft_ms'], d['ms_per_step'], e['prefill_s'], e['decode_s'], d['steady_state_decode_ratio'])"
done
