set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_tile_gpu.py -m gpu -x -q -k "paged or decode_batch" --timeout 120 --timeout-method thread > gpurun_out/pytest_r3g.log 2>&1 && tail -2 gpurun_out/pytest_r3g.log &&
timeout -k 10 200 python -u scripts/microbench.py --what prefill > gpurun_out/mb_prefill_r3c.json 2>gpurun_out/mb_prefill_r3c.err
