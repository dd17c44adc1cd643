set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_tile_gpu.py -m gpu -x -q -k "stream_k or decode_batch or prefill_dispatch" --timeout 120 --timeout-method thread > gpurun_out/pytest_r3l.log 2>&1 && tail -2 gpurun_out/pytest_r3l.log &&
timeout -k 10 300 python -u scripts/gemm_probe.py --shapes 288:152064:3584,384:152064:3584,512:152064:3584 --reps 6 --no-lib --out gpurun_out/lmhead_r3l.jsonl > gpurun_out/lmhead_r3l.log 2>&1 &&
cp githubrepostorag_amd/tuning/gemm_prefill_gfx950.json gpurun_out/gemm_prefill_gfx950.json &&
timeout -k 10 900 python -u scripts/sweep_prefill_gemm.py --models qwen2-7b --labels qkv,o,down --merge --reps 5 \
  --out gpurun_out/gemm_prefill_gfx950.json --log gpurun_out/sweep_prefill_r3l.jsonl > gpurun_out/sweep_prefill_r3l.out 2>&1
