# Multi-rank rehearsal on ONE shared GPU (gloo; RCCL refuses two ranks per device): the DP bench path
# (sharded index, per-shard top-k exchange, max over ranks, rank-0 JSON) end to end.  Ingest is skipped:
# two ranks' ingest engines do not fit one card's memory (each sizes its KV pool from free memory).
mkdir -p gpurun_out
GRAG_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 1 --warmup 1 --no-ingest \
  > gpurun_out/bench_dp2_gloo.log 2>&1
rc=$?; grep '^{' gpurun_out/bench_dp2_gloo.log | cut -c1-400; exit $rc
