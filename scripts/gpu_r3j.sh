set -o pipefail
mkdir -p gpurun_out
cp githubrepostorag_amd/tuning/gemm_prefill_gfx950.json gpurun_out/prefill_table_before.json &&
cp githubrepostorag_amd/tuning/gemm_prefill_gfx950.json gpurun_out/gemm_prefill_gfx950.json && timeout -k 10 900 python -u scripts/sweep_prefill_gemm.py --models qwen2-7b,bge-large --labels qkv,o,down,ffn1,ffn2 --merge --reps 5 \
  --out gpurun_out/gemm_prefill_gfx950.json --log gpurun_out/sweep_prefill_r3.jsonl > gpurun_out/sweep_prefill_r3.out 2>&1
