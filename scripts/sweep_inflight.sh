set -o pipefail
mkdir -p gpurun_out
for f in 4 6 3; do
  timeout -k 10 300 python -u bench.py --no-ingest --agent-jobs 0 --inflight $f > gpurun_out/inflight_$f.log 2>&1 || exit $?
  grep '^{' gpurun_out/inflight_$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($f, d['value'], d['p50_ttft_ms'], d['ms_per_step'], d['engine_per_timed_step']['decode_s'], d['engine_per_timed_step']['prefill_s'])"
done
