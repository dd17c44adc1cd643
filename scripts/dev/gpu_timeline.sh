set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_tl -o run -- \
  python3 "$R/bench.py" --steps 2 --warmup 1 --no-ingest --agent-jobs 0 $TLARGS > "$R/gpurun_out/timeline_bench.log" 2>&1 || exit 1
T=$(find /tmp/prof_tl -name "*kernel_trace.csv" | head -1)
python3 "$R/scripts/timeline_prof.py" "$T" --last-ms 2300 > "$R/gpurun_out/timeline_summary.txt" && cat "$R/gpurun_out/timeline_summary.txt"
