#!/bin/bash
# rocprofv3 kernel trace + stats over scripts/prof_decode_step.py (one decode step's graph replayed):
#   TAG=x bash scripts/profile_decode_step.sh --B 176 --ctx 1500 --split-len 1024
# stats CSV -> gpurun_out/<TAG>_dec_kernel_stats.csv, family summary on stdout.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${TAG:-dec}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
rm -rf "/tmp/prof_$T"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "/tmp/prof_$T" -o run -- \
  python3 "$R/scripts/prof_decode_step.py" "$@" > "$R/gpurun_out/${T}_dec.log" 2>&1
rc=$?
find "/tmp/prof_$T" -name "*kernel_stats.csv" -exec cp {} "$R/gpurun_out/${T}_dec_kernel_stats.csv" \;
tail -3 "$R/gpurun_out/${T}_dec.log"
[ $rc -eq 0 ] && python3 "$R/scripts/summarize_prof.py" "$R/gpurun_out/${T}_dec_kernel_stats.csv" "decode step $*"
exit $rc
