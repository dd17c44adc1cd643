set -o pipefail
mkdir -p gpurun_out
cp githubrepostorag_amd/tuning/gemm_prefill_gfx950.json gpurun_out/gemm_prefill_gfx950.json &&
timeout -k 10 900 python -u scripts/sweep_prefill_gemm.py --models qwen2-7b --labels gate_up --merge --reps 5 \
  --out gpurun_out/gemm_prefill_gfx950.json --log gpurun_out/sweep_prefill_r3n.jsonl > gpurun_out/sweep_prefill_r3n.out 2>&1
