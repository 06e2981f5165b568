#!/bin/bash
# Stall / instruction-mix breakdown of every conv3 instantiation in one bench step (SQ counters, one
# rocprofv3 pass per counter group; MI355X_MICROARCH.md rocprofv3 PMC slots).
set -o pipefail
O=gpurun_out/${TAG:-c3pmc}; mkdir -p $O
export TMPDIR=/tmp
K=${KREGEX:-conv3_kernel}
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "$K" --output-format csv -d $O/p$i -o pmc -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fp32-line > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
  python tools/pmcsum.py $O/p$i "$K" > $O/sum$i.txt 2>&1
  cat $O/sum$i.txt
done
echo done
