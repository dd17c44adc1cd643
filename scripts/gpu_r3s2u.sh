# batched sampler reset tests, then GPU busy / idle over the timed steps of a short bench (kernel trace)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
[ -n "$NOTEST" ] || timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -q \
  -k "reset_slots or sampl or engine or graph or mixed or decode" --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_rs.log 2>&1 || { tail -30 gpurun_out/pytest_rs.log; exit 1; }
tail -1 gpurun_out/pytest_rs.log
export TMPDIR=/tmp
( cd /tmp && export GRAG_TRACE_MARK=1 && timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d /tmp/tl -o run -- \
  python3 $R/bench.py --steps 2 --warmup 1 --no-ingest --agent-jobs 0 > $R/gpurun_out/tl_bench.log 2>&1 ) \
  || { tail -20 $R/gpurun_out/tl_bench.log; exit 1; }
f=$(find /tmp/tl -name "*kernel_trace.csv" | head -1)
python3 $R/scripts/timeline_prof.py $f --marker "FillFunctor<double>" > $R/gpurun_out/timeline_final.txt 2>&1
head -30 $R/gpurun_out/timeline_final.txt
