set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/w4_probe.py --reps 10 --out gpurun_out/w4_probe_r3.jsonl > gpurun_out/w4_probe_r3.log 2>&1 && echo "w4 probe ok" &&
timeout -k 10 300 python -u scripts/gemm_probe.py --shapes 288:152064:3584,320:152064:3584,384:152064:3584,448:152064:3584 --reps 8 --out gpurun_out/gemm_probe_lmhead_r3.jsonl > gpurun_out/gemm_probe_lmhead_r3.log 2>&1 && echo "lm head probe ok"
