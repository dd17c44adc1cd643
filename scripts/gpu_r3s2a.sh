# session 2: mixed-step GPU test, then serving sweeps separate vs mixed steps (no ingest / agent phases)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/pytest_mixed.log 2>&1 || { tail -20 gpurun_out/pytest_mixed.log; exit 1; }
tail -2 gpurun_out/pytest_mixed.log
for cfg in "0 16384" "1 16384" "1 4096" "1 8192"; do
  set -- $cfg
  timeout -k 10 400 python -u bench.py --no-ingest --agent-jobs 0 --steps 4 --warmup 1 --mixed $1 --max-batched-tokens $2 \
    > gpurun_out/bench_mx$1_$2.log 2>&1 || { tail -20 gpurun_out/bench_mx$1_$2.log; exit 1; }
  echo "mixed=$1 budget=$2"; grep '^{' gpurun_out/bench_mx$1_$2.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['engine_per_timed_step']
print(d['value'], d['p50_ttft_ms'], d['ms_per_step'], e['prefill_s'], e['decode_s'], e['steps'], e['decode_steps'], e.get('mixed_steps'), d['steady_state_decode_ratio'])"
done
