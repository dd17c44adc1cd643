#!/bin/bash
# PMC passes (counters with --kernel-trace only; one rocprofv3 run per counter group) over any python script:
#   TAG=name bash scripts/pmc_py.sh scripts/prof_decode_step.py --B 176 --ctx 1500
# CSVs under gpurun_out/pmc_<TAG>/p<i>; per-call averages: python scripts/pmc_dump.py gpurun_out/pmc_<TAG>
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_${TAG:-py}
mkdir -p $OUT
export TMPDIR=/tmp
SCRIPT=$R/$1
shift
cd /tmp
i=0
for P in "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA" \
         "SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
         "FETCH_SIZE TCC_HIT_sum" \
         "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 $SCRIPT "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
echo ok
