#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run -> gpurun_out/prof_<tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
TAG=${TAG:-bench}
mkdir -p gpurun_out/prof_$TAG
export TMPDIR=/tmp
cd /tmp
timeout -k 10 ${PROF_TIMEOUT:-900} rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py ${BENCH_ARGS:---steps 1 --warmup 1 --no-ingest} > $R/gpurun_out/prof_$TAG/bench_stdout.log 2>&1
rc=$?
echo "rc=$rc"
# the per-dispatch trace is large; keep only the summaries
find $R/gpurun_out/prof_$TAG -name "*kernel_trace.csv" -delete
tail -5 $R/gpurun_out/prof_$TAG/bench_stdout.log
f=$(find $R/gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 $R/scripts/summarize_prof.py "$f" 40
exit $rc
