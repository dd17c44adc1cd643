# same-box A/B of the Python GIL switch interval (engine thread vs the retrieval prefetch thread)
set -o pipefail
mkdir -p gpurun_out
for si in 0 0.0005 0.002 0 0.0005 0.002; do
  timeout -k 10 400 python -u bench.py --no-ingest --agent-jobs 0 --steps 8 --warmup 1 --switch-interval $si \
    > gpurun_out/ab_switch_$si.log 2>&1 || { tail -20 gpurun_out/ab_switch_$si.log; exit 1; }
  echo "si=$si $(grep '^{' gpurun_out/ab_switch_$si.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['engine_per_timed_step']
print(d['value'], d['p50_ttft_ms'], d['ms_per_step'], e['prefill_s'], e['decode_s'], e['host_sched_s'])")"
done
