# Multi-rank rehearsal on ONE shared GPU (gloo; RCCL refuses two ranks per device): the driver's own
# command form (`python bench.py --gpus 2`, ranks self-spawned) through the DP bench path end to end —
# sharded index, per-shard top-k exchange, max over ranks, rank-0 JSON, and the agent phase through one
# front door over the two sharded replicas.  Ingest is skipped: two ranks' ingest engines do not fit one
# card's memory (each sizes its KV pool from free memory).
mkdir -p gpurun_out
GRAG_DIST_BACKEND=gloo timeout -k 10 900 python bench.py --gpus 2 --steps 2 --warmup 1 --no-ingest \
  --agent-jobs 64 > gpurun_out/bench_dp2_gloo.log 2>&1
rc=$?; grep '^{' gpurun_out/bench_dp2_gloo.log | cut -c1-600; exit $rc
