set -e
TAG=g192bal ARGS="--shape gate_up --M 192 --plan 12,5,2,1,256" bash scripts/pmc_dec.sh
TAG=g192tile ARGS="--shape gate_up --M 192 --plan tile" bash scripts/pmc_dec.sh
TAG=g128bal ARGS="--shape gate_up --M 128 --plan 8,5,2,1,256" bash scripts/pmc_dec.sh
