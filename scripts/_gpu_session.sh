mkdir -p gpurun_out
timeout -k 10 300 python -m pytest -q -x tests/test_engine_gpu.py > gpurun_out/te.log 2>&1 || { tail -30 gpurun_out/te.log; exit 1; }
tail -1 gpurun_out/te.log
for cfg in "2 8" "3 8" "3 1" "2 4"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --no-ingest --inflight $1 --arrival-groups $2 > gpurun_out/bT_$1_$2.log 2>&1 || { tail -20 gpurun_out/bT_$1_$2.log; exit 1; }
  python - gpurun_out/bT_$1_$2.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e = d["engine"]
print(sys.argv[1], d["value"], "q/s  p50", d["p50_ttft_ms"], "ms  step", d["ms_per_step"], "prefill_s", e["prefill_s"],
      "decode_s", e["decode_s"], "wait", e["decode_wait_s"], "steps", e["steps"], "capt", e["graph_captures"])
PY
done
timeout -k 10 300 python scripts/bench_prefill_gemm.py --M 4096,6912,8192,16384 --out gpurun_out/prefill_gemm.json > gpurun_out/pg.log 2>&1 || exit 1
grep -o "^[a-z_]* [0-9]* .*TFLOP_s': [0-9.]*" gpurun_out/pg.log | sed -E "s/\{'engine_linear.*TFLOP_s'/TF/"
