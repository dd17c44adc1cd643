# session 2: mixed-step GPU test, then serving sweeps separate vs mixed steps (no ingest / agent phases)
# CFGS="0_16384 1_4096" STEPS=8 NOTEST=1 bash scripts/gpu_r3s2a.sh   (mixed_budget pairs)
set -o pipefail
mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_mixed.log 2>&1 || { tail -20 gpurun_out/pytest_mixed.log; exit 1; }
  tail -2 gpurun_out/pytest_mixed.log
fi
for cfg in ${CFGS:-0_16384 1_16384 1_4096 1_8192}; do
  mx=${cfg%_*}; bud=${cfg#*_}
  timeout -k 10 400 python -u bench.py --no-ingest --agent-jobs 0 --steps ${STEPS:-4} --warmup 1 --mixed $mx \
    --max-batched-tokens $bud ${EXTRA:-} > gpurun_out/bench_mx${mx}_${bud}${TAG:-}.log 2>&1 \
    || { tail -20 gpurun_out/bench_mx${mx}_${bud}${TAG:-}.log; exit 1; }
  echo "mixed=$mx budget=$bud"; grep '^{' gpurun_out/bench_mx${mx}_${bud}${TAG:-}.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['engine_per_timed_step']
print('qps', d['value'], 'ttft', d['p50_ttft_ms'], 'ms', d['ms_per_step'], 'pre_s', e['prefill_s'], 'dec_s', e['decode_s'], 'steps', e['steps'], 'dsteps', e['decode_steps'], 'mixed', e.get('mixed_steps'), 'ptok', e['prefill_tokens'], 'dtok', e['decode_tokens'], 'ratio', d['steady_state_decode_ratio'])"
done
