#!/bin/bash
# rocprofv3 kernel trace + stats over a short bench (no PMC counters: those go in their own passes,
# scripts/pmc_gemm.sh).  Only the stats CSVs are copied to gpurun_out/ (the full trace is large).
#   bash scripts/profile_bench.sh [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_bench -o run -- \
  python3 "$R/bench.py" --steps 2 --warmup 1 --no-ingest --agent-jobs 0 "$@" > "$R/gpurun_out/profile_bench.log" 2>&1
rc=$?
find /tmp/prof_bench -name "*kernel_stats.csv" -exec cp {} "$R/gpurun_out/" \;
[ $rc -eq 0 ] && python3 "$R/scripts/summarize_prof.py" "$R/gpurun_out/run_kernel_stats.csv" "rocprofv3 kernel stats: bench.py --steps 2 --warmup 1 --no-ingest --agent-jobs 0 $*"
exit $rc
