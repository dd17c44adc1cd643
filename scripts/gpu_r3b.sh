set -o pipefail
mkdir -p gpurun_out
timeout -k 10 180 python -u scripts/dev/w4_diag.py --run --reps 3 > gpurun_out/w4_diag2.log 2>&1
echo "w4 diag rc=$?"
S=""
for M in 320 384 448 512; do S="$S,$M:4608:3584,$M:3584:3584,$M:37888:3584:silu,$M:3584:18944"; done
S="${S#,},512:152064:3584,256:152064:3584,128:152064:3584"
timeout -k 10 600 python -u scripts/gemm_probe.py --shapes "$S" --reps 10 --out gpurun_out/gemm_probe_r3.jsonl > gpurun_out/gemm_probe_r3.log 2>&1
echo "probe rc=$?"
grep '"best": true' gpurun_out/gemm_probe_r3.jsonl | cut -c1-200
