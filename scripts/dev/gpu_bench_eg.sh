set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 --no-ingest --agent-jobs 0 --switch-interval 0.0005 > gpurun_out/bench_eg1si.log 2>&1 || exit 1
GRAG_ENCODER_GRAPHS=0 timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 --no-ingest --agent-jobs 0 > gpurun_out/bench_eg0.log 2>&1 || exit 1
timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 --no-ingest --agent-jobs 0 > gpurun_out/bench_eg1.log 2>&1
