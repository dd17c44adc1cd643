set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_tile_gpu.py -x -q --timeout 120 --timeout-method thread -k "stream_k" > gpurun_out/tile_tests.log 2>&1
timeout -k 10 500 python -u scripts/bench_gemm_tile.py --shapes prefill --prefill-ms 8192,16384 --reps 15 --out gpurun_out/gemm_tile_ab_tail.jsonl > gpurun_out/tile8k.log 2>&1
