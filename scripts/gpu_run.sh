#!/bin/bash
# One parametrised GPU session runner (replaces round 3's per-session scripts/gpu_r3*.sh).
#
#   TAG=r4a bash scripts/gpu_run.sh STEP [STEP ...]
#
# Steps (each under its own time limit, logs in gpurun_out/<TAG>_<step>.log):
#   tests[=SEL]      pytest -m gpu over SEL (default: tests)              (600 s)
#   smoke            __graft_entry__.smoke()                              (300 s)
#   bench[=ARGS]     python bench.py ARGS (',' separates args)            (900 s)
#   preset=cN        python bench.py --preset cN (BASELINE config N)      (900 s)
#   dp2              shared-GPU DP rehearsal: bench --gpus 2, gloo, both ranks on cuda:0
#   tp2              shared-GPU TP rehearsal: bench --gpus 2 --tp 2 (IPC all-reduce + vocab-parallel
#                    sampler in the decode graphs, lockstep ingest and agent)
#   c4tp8            BASELINE config 4's per-rank shapes rehearsed on ONE GPU: Qwen2-72B at TP=8 as 8 rank
#                    processes sharing the card (18 GB of weights each), small batch / index / KV; ranks
#                    sharing a device run process-group (gloo-staged) collectives and eager decode, so
#                    the agent phase is one job (4 took > 400 s, profiles/rehearse_c4tp8_shared_gpu_r5.log)
#   sweep=LEVELS     bench with --agent-sweep LEVELS (agent saturation curve); SWEEP_ARGS=a,b,.. extra bench args
#   prof             rocprofv3 --kernel-trace --stats over a 2-step bench (scripts/profile_bench.sh)
#   mb=WHAT          scripts/microbench.py --what WHAT (json in gpurun_out/<TAG>_mb_WHAT.json)
#   profdec=ARGS     rocprofv3 kernel stats of one decode step (scripts/profile_decode_step.sh ARGS)  (400 s)
#   pmcdec=ARGS      PMC passes over scripts/prof_dec.py ARGS (scripts/pmc_dec.sh; csv under gpurun_out/pmc_<TAG>_pmcN)
#   pmcpy=SCRIPT,ARGS PMC passes over any python script (scripts/pmc_py.sh; summary: scripts/pmc_dump.py)
#   py=SCRIPT,ARGS   python -u SCRIPT ARGS (',' separates args; log gpurun_out/<TAG>_py<i>.log)  (600 s)
#   envpy=A=1+B=2,SCRIPT,ARGS  the same with environment variables ('+' separates them)
#
# A step that exits 0 or 1 (a clean Python failure) lets the next one run; a fault, abort, segfault or
# time limit (124 / 134 / 137 / 139) ends the session there (no more GPU work after a GPU fault).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-run}
worst=0

run() {  # run LIMIT NAME CMD...
  local lim=$1 name=$2
  shift 2
  local log="gpurun_out/${TAG}_${name}.log"
  echo "== $name: $*"
  timeout -k 10 "$lim" "$@" > "$log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -E '^\{' "$log" | cut -c1-900 || true
  grep -E "passed|failed|error|serving|agent e2e|ingest:|smoke ok|Traceback" "$log" | tail -6 || true
  [ $rc -ne 0 ] && tail -25 "$log"
  [ $rc -gt $worst ] && worst=$rc
  case $rc in 0|1|2) return 0 ;; *) echo "== stopping: $name ended with $rc"; exit $rc ;; esac
}

npy=0
npd=0
REH="--steps 2 --warmup 1 --kv-cache-gb 48 --ingest-kv-gb 24 --ingest-files 48 --ingest-ref-cap-files 0 --agent-jobs 64"
for step in "$@"; do
  key=${step%%=*}
  val=""
  [[ "$step" == *=* ]] && val=${step#*=}
  case $key in
    tests) run 600 "tests" python -u -m pytest ${val:-tests} -m gpu -x -q --timeout 240 --timeout-method thread ;;
    smoke) run 300 smoke python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run 900 bench python -u bench.py ${val//,/ } ;;
    preset) run 900 "preset_$val" python -u bench.py --preset "$val" --out "gpurun_out/${TAG}_preset_$val.json" ;;
    dp2) run 900 dp2 env GRAG_DIST_BACKEND=gloo python -u bench.py --gpus 2 $REH ${val//,/ } ;;
    tp2) run 900 tp2 env GRAG_DIST_BACKEND=gloo python -u bench.py --gpus 2 --tp 2 $REH ${val//,/ } ;;
    c4tp8) run 1100 c4tp8 env GRAG_DIST_BACKEND=gloo python -u bench.py --gpus 8 --tp 8 --model qwen2-72b \
             --index-size 2000000 --nlist 1024 --nprobe 32 --batch 8 --inflight 2 --arrival-groups 2 --steps 2 \
             --warmup 1 --kv-cache-gb 6 --max-batched-tokens 480 --no-ingest --agent-jobs 1 \
             --agent-concurrency 1 --serving-steps 0 --prompt-len 256 --gen-len 16 --agent-gen-len 8 \
             --agent-synth-len 16 --low-load 0 --recall-queries 8 --heartbeat 30 ${val//,/ } ;;
    sweep) run 1100 sweep python -u bench.py --no-ingest --agent-sweep "${val:-64,256,512,1024}" --steps 2 --warmup 1 \
             ${SWEEP_ARGS//,/ } ;;
    prof) run 700 prof bash scripts/profile_bench.sh ;;
    profdec) npd=$((npd+1)); run 400 "profdec$npd" env TAG="${TAG}_$npd" bash scripts/profile_decode_step.sh ${val//,/ } ;;
    pmcdec) run 400 "pmcdec_$npy" env TAG="${TAG}_pmc$npy" ARGS="${val//,/ }" bash scripts/pmc_dec.sh; npy=$((npy+1)) ;;
    pmcpy) run 600 "pmcpy_$npy" env TAG="${TAG}_pmcpy$npy" bash scripts/pmc_py.sh ${val//,/ }; npy=$((npy+1)) ;;
    py) npy=$((npy+1)); run 600 "py$npy" python -u ${val//,/ } ;;
    envpy) npy=$((npy+1)); ev=${val%%,*}; rest=${val#*,}; run 600 "py$npy" env ${ev//+/ } python -u ${rest//,/ } ;;
    mb) run 400 "mb_$val" python -u scripts/microbench.py --what "$val" --out "gpurun_out/${TAG}_mb_$val.json" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
exit $worst
