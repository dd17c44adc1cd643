# same-box A/B: decode through hipGraph replays vs eager launches (depth 16, 1024-row 1-step windows)
set -o pipefail
mkdir -p gpurun_out
for arm in graph eager graph eager; do
  extra=""; [ $arm = eager ] && extra="--no-graph"
  timeout -k 10 400 python -u bench.py --no-ingest --agent-jobs 0 --steps 8 --warmup 1 $extra \
    > gpurun_out/ab_graph_$arm.log 2>&1 || { tail -20 gpurun_out/ab_graph_$arm.log; exit 1; }
  echo "$arm $(grep '^{' gpurun_out/ab_graph_$arm.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['engine_per_timed_step']
print(d['value'], d['p50_ttft_ms'], d['ms_per_step'], e['prefill_s'], e['decode_s'], e['decode_steps'], e['graph_replays'])")"
done
