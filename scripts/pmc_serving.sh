#!/bin/bash
# PMC passes (counters with --kernel-trace only; no sys/runtime/hip traces) over scripts/pmc_serving.py at
# the serving bench's operating points -> gpurun_out/pmc_serving/<mode>/p<i>, then one summary per mode.
# Per-pass counter budget (MI355X_MICROARCH.md): SQ <= 8, TCC <= 4 (FETCH_SIZE takes 3, WRITE_SIZE 2), GRBM <= 2.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_serving
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for MODE in "gemm --M 4096" "gemm --M 7104" "decode"; do
  TAGN=$(echo $MODE | tr -d ' -')
  i=0
  for P in "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE FETCH_SIZE" \
           "WRITE_SIZE SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/$TAGN/p$i -o run -- \
      python3 $R/scripts/pmc_serving.py --mode $MODE > $OUT/$TAGN.p$i.log 2>&1 || { echo "$TAGN pass $i failed"; tail -5 $OUT/$TAGN.p$i.log; exit 1; }
    find $OUT/$TAGN/p$i -name "*kernel_trace.csv" -size +20M -delete
    echo "$TAGN pass $i ok"
  done
  python3 $R/scripts/summarize_pmc.py $OUT/$TAGN > $OUT/$TAGN.summary.txt && cat $OUT/$TAGN.summary.txt
done
