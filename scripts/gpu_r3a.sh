set -o pipefail
mkdir -p gpurun_out
timeout -k 10 180 python -u scripts/dev/w4_diag.py --run --reps 4 > gpurun_out/w4_diag.log 2>&1
echo "w4 diag rc=$?"; grep -c max_rel_err gpurun_out/w4_diag.log
bash scripts/gpu_quick.sh tests r3v1
