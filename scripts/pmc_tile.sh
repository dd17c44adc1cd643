#!/bin/bash
# PMC passes over scripts/prof_tile.py (counters only with --kernel-trace; no sys/runtime traces).
# ARGS="--shape gate_up --M 7104" TAG=tile_gu bash scripts/pmc_tile.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_${TAG:-tile}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 python3 $R/scripts/prof_tile.py ${ARGS} > $OUT/wall.log 2>&1 || { echo "wall run failed"; tail -5 $OUT/wall.log; exit 1; }
cat $OUT/wall.log
i=0
for P in "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" \
         "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU" \
         "FETCH_SIZE TCC_HIT_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 $R/scripts/prof_tile.py ${ARGS} --reps 20 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
echo ok
