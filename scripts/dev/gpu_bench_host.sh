set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --no-ingest --agent-jobs 0 --pysample 0.5 > gpurun_out/bench_host.log 2>&1
