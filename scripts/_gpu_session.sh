mkdir -p gpurun_out
for cfg in "3 8" "3 4" "4 8" "3 1"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --no-ingest --inflight $1 --arrival-groups $2 > gpurun_out/bS_$1_$2.log 2>&1 || { tail -20 gpurun_out/bS_$1_$2.log; exit 1; }
  python - gpurun_out/bS_$1_$2.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e = d["engine_per_timed_step"]
print(sys.argv[1], d["value"], "q/s  p50", d["p50_ttft_ms"], "ms  step", d["ms_per_step"], d["phase_ms_per_step"])
print("   per step:", {k: e[k] for k in ("prefill_s", "decode_s", "decode_wait_s", "steps", "graph_replays", "graph_captures", "decode_steps")})
PY
done
