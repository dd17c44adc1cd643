set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_tile_gpu.py tests/test_hf_parity.py tests/test_linear_dispatch.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r3i.log 2>&1 && tail -2 gpurun_out/pytest_r3i.log &&
bash scripts/ab_lib.sh "python -u scripts/gemm_probe.py --shapes 7104:37888:3584:silu,7104:3584:18944,7104:4608:3584 --reps 8" gemm 2
