#!/bin/bash
# Stall breakdown of the 64->64 @512^2 weight gradient (SQ counters, one pass per group).
set -o pipefail
O=gpurun_out/wpmc; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/wgrad_one.py > $O/time.txt 2>&1 || { cat $O/time.txt; exit 1; }
cat $O/time.txt
rocprofv3 -L > $O/counters.txt 2>&1 || true
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex 'wgrad2_kernel' --output-format csv -d $O/p$i -o pmc -- python tools/wgrad_one.py 4 512 512 64 64 4 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; }
  python tools/pmcsum.py $O/p$i wgrad2 2>/dev/null || true
done
echo done
