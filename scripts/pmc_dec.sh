#!/bin/bash
# PMC passes over scripts/prof_dec.py (counters with --kernel-trace only; one pass per counter group).
# usage: TAG=name ARGS="--shape gate_up --M 192 --plan 12,5,2,1,256" bash scripts/pmc_dec.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_${TAG:-dec}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for P in "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA" \
         "SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
         "FETCH_SIZE TCC_HIT_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 $R/scripts/prof_dec.py ${ARGS} > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
echo ok
