#!/bin/bash
# Bare-metal launcher for one 8 x MI355X node (no Kubernetes):
#   ./deploy/launch_node.sh serve    -> one front door on :8000 (one /rag/jobs + SSE endpoint, one queue)
#                                       over NGPU replica processes, one per GPU (service/cluster.py)
#   ./deploy/launch_node.sh ingest   -> data-parallel ingest: NGPU rank processes (one per GPU) split the
#                                       repositories (--repos ...), then write NGPU shard snapshots
#                                       $INDEX_DIR/shard-r-of-NGPU that `serve` loads one per replica
#                                       (INDEX_SHARDING=shard, the default); NGPU=1: one process, one snapshot
#   ./deploy/launch_node.sh bench N  -> the multi-GPU bench (N rank processes, one per GPU, RCCL;
#                                       bench.py spawns them itself, no launcher)
set -euo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
NGPU=${NGPU:-8}
case "${1:-serve}" in
  serve)
    GPUS=$(seq -s, 0 $((NGPU - 1))) exec python -m githubrepostorag_amd serve --replicas "$NGPU" --port "${PORT:-8000}" ;;
  ingest)
    python -m githubrepostorag_amd ingest --dp "$NGPU" "${@:2}" ;;
  bench)
    N=${2:-$NGPU}
    python bench.py --gpus "$N" "${@:3}" ;;
  *) echo "usage: $0 serve|ingest|bench [N]"; exit 2 ;;
esac
