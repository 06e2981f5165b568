#!/bin/bash
# PMC breakdown of the 1->64 first-layer kernels (smallcin fwd / wgrad) over two bench steps: SQ issue and
# stall counters, then HBM bytes (FETCH_SIZE, WRITE_SIZE) in their own passes.
set -o pipefail
O=gpurun_out/scpmc; mkdir -p $O
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex 'smallcin' --output-format csv -d $O/p$i -o pmc -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
  python tools/pmcsum.py $O/p$i smallcin
done
echo done
