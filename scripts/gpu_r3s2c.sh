# tile GEMM counters at the bench's prefill operating point (gate/up SwiGLU and down_proj at 7104 rows)
set -o pipefail
ARGS="--shape gate_up --M 7104" TAG=tile_gu bash scripts/pmc_tile.sh && \
ARGS="--shape down --M 7104" TAG=tile_down bash scripts/pmc_tile.sh && \
ARGS="--shape qkv --M 7104" TAG=tile_qkv bash scripts/pmc_tile.sh
