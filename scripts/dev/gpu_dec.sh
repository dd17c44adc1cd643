set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_tile_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dec_tests.log 2>&1
timeout -k 10 600 python -u scripts/bench_gemm_decode.py --ms 48,64,96,128,160,192,224,256 --reps 21 --dispatch --out gpurun_out/gemm_decode_dispatch_r2.jsonl > gpurun_out/dec_bench.log 2>&1
