# same-box A/B: ingest with separate prefill / decode steps vs mixed steps (decode rows in prefill steps)
set -o pipefail
mkdir -p gpurun_out
for mx in 0 1 0 1; do
  timeout -k 10 400 python -u bench.py --steps 1 --warmup 0 --agent-jobs 0 --ingest-ref-cap-files 0 --ingest-mixed $mx \
    > gpurun_out/ab_ingest_mx$mx.log 2>&1 || { tail -20 gpurun_out/ab_ingest_mx$mx.log; exit 1; }
  echo "mixed=$mx $(grep '^{' gpurun_out/ab_ingest_mx$mx.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['ingest_stage_s']['engine']
print(d['ingest_docs_per_s'], e['prefill_s'], e['decode_s'], e['decode_steps'], e['mixed_steps'], e['steps'])")"
done
