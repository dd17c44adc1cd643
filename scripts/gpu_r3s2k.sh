# same-box A/B of the prefill dispatch tables: current (r3c re-sweep) vs the previous (r3b) table
set -o pipefail
mkdir -p gpurun_out
for arm in new old new old; do
  if [ $arm = old ]; then export GRAG_PREFILL_TABLE=scripts/dev/prefill_table_r3b.json; else export GRAG_PREFILL_TABLE=1; fi
  timeout -k 10 300 python -u bench.py --no-ingest --agent-jobs 0 --steps 4 --warmup 1 > gpurun_out/ab_table_$arm.log 2>&1 \
    || { tail -20 gpurun_out/ab_table_$arm.log; exit 1; }
  echo "$arm $(grep '^{' gpurun_out/ab_table_$arm.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['engine_per_timed_step']
print(d['value'], d['p50_ttft_ms'], d['ms_per_step'], e['prefill_s'], e['decode_s'])")"
done
