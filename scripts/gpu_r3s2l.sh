# same-box A/B: retrieval side stream at high vs normal priority (search kernels vs engine GEMMs)
set -o pipefail
mkdir -p gpurun_out
for arm in high normal high normal; do
  export GRAG_SIDE_PRIORITY=$arm
  timeout -k 10 300 python -u bench.py --no-ingest --agent-jobs 0 --steps 4 --warmup 1 > gpurun_out/ab_prio_$arm.log 2>&1 \
    || { tail -20 gpurun_out/ab_prio_$arm.log; exit 1; }
  echo "$arm $(grep '^{' gpurun_out/ab_prio_$arm.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['engine_per_timed_step']; ph=d['phase_ms_per_step']
print(d['value'], d['p50_ttft_ms'], d['ms_per_step'], e['prefill_s'], e['decode_s'], ph['search'])")"
done
