set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 --no-ingest --agent-jobs 0 --gc-freeze 0 > gpurun_out/bench_gc0.log 2>&1 || exit 1
timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 --no-ingest --agent-jobs 0 --gc-freeze 1 > gpurun_out/bench_gc1.log 2>&1
