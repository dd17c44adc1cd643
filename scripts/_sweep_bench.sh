#!/bin/bash
# sweep the serving-mode knobs of bench.py (in-flight batches x arrival groups)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
for cfg in ${CFGS:-2x8 3x8 4x8 3x16 4x16}; do
  set -- ${cfg/x/ }
  timeout -k 10 300 python bench.py --no-ingest --steps 3 --inflight $1 --arrival-groups $2 ${EXTRA} > gpurun_out/bS_$1_$2.log 2>&1 || { tail -20 gpurun_out/bS_$1_$2.log; exit 1; }
  python - gpurun_out/bS_$1_$2.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e = d["engine_per_timed_step"]
print(sys.argv[1], d["value"], "q/s  p50", d["p50_ttft_ms"], "ms  step", d["ms_per_step"], d["phase_ms_per_step"])
print("   prefetch:", d.get("retrieval_prefetch"), "per step:", {k: e[k] for k in ("prefill_s", "decode_s", "decode_wait_s", "steps", "graph_replays", "graph_captures", "decode_steps", "decode_tokens")})
PY
done
