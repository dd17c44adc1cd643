#!/bin/bash
# rocprofv3 PMC passes (one run per pass, counters with --kernel-trace only:
# no sys/runtime/hip traces) over scripts/pmc_kernels.py -> gpurun_out/pmc_kernels
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_kernels
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for P in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR FETCH_SIZE" \
         "WRITE_SIZE SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 $R/scripts/pmc_kernels.py > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  find $OUT/p$i -name "*kernel_trace.csv" -size +20M -delete
  echo "pass $i ok"
done
python3 $R/scripts/summarize_pmc.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
