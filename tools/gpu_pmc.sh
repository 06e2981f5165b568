#!/bin/bash
# HBM traffic of the probed conv kernel: separate FETCH_SIZE / WRITE_SIZE passes (MI355X_MICROARCH.md
# HBM/rocprofv3 section), plus the conv3 ablation timings.  Each GPU step has its own time limit.
set -o pipefail
O=gpurun_out/${TAG:-pmc}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/conv_ablate.py ${ABL:-200,201,202,203,208,215,216,232} > $O/ablate.txt 2>&1 || { echo "ablate failed"; tail -20 $O/ablate.txt; exit 1; }
cat $O/ablate.txt
i=0
for set in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex 'conv3_kernel' --output-format csv -d $O/pmc$i -o pmc -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pmc$i.log; exit 1; }
  python tools/pmcsum.py $O/pmc$i conv3_kernel
done
echo done
