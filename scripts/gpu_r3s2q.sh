# same-box A/B of the in-flight depth (live sequences = 64 x D)
set -o pipefail
mkdir -p gpurun_out
for d in 8 12 16 8 12 16; do
  timeout -k 10 400 python -u bench.py --no-ingest --agent-jobs 0 --steps 8 --warmup 1 --inflight $d \
    > gpurun_out/ab_depth_$d.log 2>&1 || { tail -20 gpurun_out/ab_depth_$d.log; exit 1; }
  echo "D=$d $(grep '^{' gpurun_out/ab_depth_$d.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['engine_per_timed_step']
print(d['value'], d['p50_ttft_ms'], d['ms_per_step'], e['prefill_s'], e['decode_s'], e['decode_steps'], d['steady_state_decode_ratio'])")"
done
