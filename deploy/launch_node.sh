#!/bin/bash
# Bare-metal launcher for one 8 x MI355X node (no Kubernetes):
#   ./deploy/launch_node.sh serve    -> one API+engine process per GPU on ports 8000..8007
#   ./deploy/launch_node.sh ingest   -> ingest on GPU 0, snapshot to $INDEX_DIR
#   ./deploy/launch_node.sh bench N  -> the multi-GPU bench (torchrun, one rank per GPU, RCCL)
set -euo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
NGPU=${NGPU:-8}
case "${1:-serve}" in
  serve)
    for i in $(seq 0 $((NGPU - 1))); do
      HIP_VISIBLE_DEVICES=$i python -m githubrepostorag_amd serve --port $((8000 + i)) > "serve_$i.log" 2>&1 &
    done
    wait ;;
  ingest)
    HIP_VISIBLE_DEVICES=0 python -m githubrepostorag_amd ingest "${@:2}" ;;
  bench)
    N=${2:-$NGPU}
    python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
      --master-port "${MASTER_PORT:-29511}" bench.py --gpus "$N" "${@:3}" ;;
  *) echo "usage: $0 serve|ingest|bench [N]"; exit 2 ;;
esac
