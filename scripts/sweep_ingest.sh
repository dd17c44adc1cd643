# GPU: ingest docs/s by ingest-engine concurrency and mixed prefill/decode steps (serving phase skipped
# to a minimum: 1 step, no agent phase).  Usage: bash scripts/sweep_ingest.sh
set -o pipefail
mkdir -p gpurun_out
for cfg in "256 0" "512 0" "256 1" "512 1"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --inflight 1 --agent-jobs 0 --ingest-seqs $1 --ingest-mixed $2 \
    > gpurun_out/ingest_s$1_m$2.log 2>&1 || exit $?
  grep '^{' gpurun_out/ingest_s$1_m$2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); st=d['ingest_stage_s']; e=st['engine']; print('seqs $1 mixed $2', d['ingest_docs_per_s'], {k: st[k] for k in ('file_summaries','module_summaries','catalog','code_nodes','repo_summaries')}, e['prefill_s'], e['decode_s'], e['mixed_steps'], e['decode_steps'])"
done
