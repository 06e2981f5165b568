#!/bin/bash
# SQ counters of conv5 (full and bare-loop ablation) on the 64->64 layers: one rocprofv3 pass per group
set -o pipefail
O=gpurun_out/${TAG:-r03j}; mkdir -p $O
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS" "SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "conv5_kernel" --output-format csv -d $O/p$i -o pmc -- python tools/conv4_ablate.py 0,8,31 --conv5 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
  python tools/pmcsum.py $O/p$i conv5_kernel > $O/sum$i.txt 2>&1
  cat $O/sum$i.txt
done
echo done
