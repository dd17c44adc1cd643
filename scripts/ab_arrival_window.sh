# GPU A/B of the runner's arrival-aware decode window on the bench's agent e2e phase (same box).
set -o pipefail
mkdir -p gpurun_out
for w in 0 2 0 2; do
  GRAG_ARRIVAL_WINDOW=$w timeout -k 10 400 python -u bench.py --no-ingest --steps 2 > gpurun_out/ab_aw_$w.log 2>&1 || exit $?
  grep '^{' gpurun_out/ab_aw_$w.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); a=d['agent_e2e']; print('window $w', d['value'], a['jobs_per_s'], a['e2e_ttft_p50_ms'], a['e2e_ttft_p90_ms'], a['job_latency_p50_ms'])"
done
