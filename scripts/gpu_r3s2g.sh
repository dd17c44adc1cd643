# session 2 combined pass: new GPU tests, decode-step profile, full GPU suite, default bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_cluster_gpu.py -m gpu -x -q \
  -k "rope or splitk or front_door" --timeout 300 --timeout-method thread > gpurun_out/pytest_new.log 2>&1 \
  || { tail -40 gpurun_out/pytest_new.log; exit 1; }
tail -2 gpurun_out/pytest_new.log
timeout -k 10 300 python -u scripts/prof_decode_step.py --B 512 --ctx 1100 > gpurun_out/dec_step.log 2>&1 || { tail -20 gpurun_out/dec_step.log; exit 1; }
tail -1 gpurun_out/dec_step.log
( export TMPDIR=/tmp; cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_dec -o run -- \
  python3 $R/scripts/prof_decode_step.py --B 512 --ctx 1100 --reps 20 > $R/gpurun_out/dec_step_prof.log 2>&1 ) || { tail -20 $R/gpurun_out/dec_step_prof.log; exit 1; }
find /tmp/prof_dec -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/dec_kernel_stats.csv \;
bash scripts/gpu_quick.sh tests s2
