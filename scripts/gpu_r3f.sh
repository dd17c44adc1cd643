set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_hf_parity.py tests/test_w4.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r3f.log 2>&1 && tail -3 gpurun_out/pytest_r3f.log &&
timeout -k 10 900 python -u bench.py > gpurun_out/bench_r3f.log 2>&1 && grep "ingest\|serving:" gpurun_out/bench_r3f.log &&
timeout -k 10 900 python -u bench.py --quant w4 > gpurun_out/bench_r3f_w4.log 2>&1 && grep "ingest\|serving:" gpurun_out/bench_r3f_w4.log
