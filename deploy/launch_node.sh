#!/bin/bash
# Bare-metal launcher for one 8 x MI355X node (no Kubernetes):
#   ./deploy/launch_node.sh serve    -> one front door on :8000 (one /rag/jobs + SSE endpoint, one queue)
#                                       over NGPU replica processes, one per GPU (service/cluster.py)
#   ./deploy/launch_node.sh ingest   -> ingest on GPU 0, snapshot to $INDEX_DIR
#   ./deploy/launch_node.sh bench N  -> the multi-GPU bench (torchrun, one rank per GPU, RCCL)
set -euo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
NGPU=${NGPU:-8}
case "${1:-serve}" in
  serve)
    GPUS=$(seq -s, 0 $((NGPU - 1))) exec python -m githubrepostorag_amd serve --replicas "$NGPU" --port "${PORT:-8000}" ;;
  ingest)
    HIP_VISIBLE_DEVICES=0 python -m githubrepostorag_amd ingest "${@:2}" ;;
  bench)
    N=${2:-$NGPU}
    python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
      --master-port "${MASTER_PORT:-29511}" bench.py --gpus "$N" "${@:3}" ;;
  *) echo "usage: $0 serve|ingest|bench [N]"; exit 2 ;;
esac
