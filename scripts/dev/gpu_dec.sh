set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_tile_gpu.py -x -q --timeout 120 --timeout-method thread -k "decode" > gpurun_out/dec_tests.log 2>&1
timeout -k 10 600 python -u scripts/bench_gemm_decode.py --ms 128,192,256 --splits 1,2,3,5,7,9,14 --reps 21 --packed --out gpurun_out/gemm_decode_ab_v6.jsonl > gpurun_out/dec_bench.log 2>&1
