set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 --no-ingest --agent-jobs 0 --prefetch 1 > gpurun_out/bench_pf1.log 2>&1 || exit 1
timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 --no-ingest --agent-jobs 0 --prefetch 0 > gpurun_out/bench_pf0.log 2>&1
