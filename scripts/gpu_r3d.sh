set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/w4_probe.py --graph --reps 8 --ms 1,16,32,64,96,128,192,256 --out gpurun_out/w4_probe_graph_r3.jsonl > gpurun_out/w4_probe_graph_r3.log 2>&1 && echo "w4 graph probe ok"
