# K-aligned tail splits: stream-K tests, then a re-sweep of the Qwen2-7B prefill shapes (merged into the table)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_tile_gpu.py -m gpu -x -q -k "stream_k" --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_sk.log 2>&1 || { tail -30 gpurun_out/pytest_sk.log; exit 1; }
tail -2 gpurun_out/pytest_sk.log
timeout -k 10 900 python -u scripts/sweep_prefill_gemm.py --models qwen2-7b --merge --mmin ${MMIN:-384} \
  --mmax ${MMAX:-16256} --log gpurun_out/sweep_prefill_r3c.jsonl > gpurun_out/sweep_prefill_r3c.out 2>&1 \
  || { tail -20 gpurun_out/sweep_prefill_r3c.out; exit 1; }
tail -3 gpurun_out/sweep_prefill_r3c.out
cp githubrepostorag_amd/tuning/gemm_prefill_gfx950.json gpurun_out/gemm_prefill_gfx950.json
