# same-box A/B of the arrival grouping at depth 16 (queries per arrival = 64 / A)
set -o pipefail
mkdir -p gpurun_out
for a in 4 8 16 4 8 16; do
  timeout -k 10 400 python -u bench.py --no-ingest --agent-jobs 0 --steps 8 --warmup 1 --arrival-groups $a \
    > gpurun_out/ab_arrival_$a.log 2>&1 || { tail -20 gpurun_out/ab_arrival_$a.log; exit 1; }
  echo "A=$a $(grep '^{' gpurun_out/ab_arrival_$a.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['engine_per_timed_step']
print(d['value'], d['p50_ttft_ms'], d['ms_per_step'], e['prefill_s'], e['decode_s'], e['steps'], e['decode_steps'], d['steady_state_decode_ratio'])")"
done
