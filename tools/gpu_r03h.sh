#!/bin/bash
# host enqueue (eager vs HIP-graph replay) and the per-kernel profile of the bench step
set -o pipefail
O=gpurun_out/${TAG:-r03h}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/cpu_overhead.py > $O/cpu_overhead.txt 2>&1 || { echo "cpu_overhead failed"; tail -20 $O/cpu_overhead.txt; exit 1; }
cat $O/cpu_overhead.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32-line > $O/trace.log 2>&1 || { echo "trace failed"; tail -20 $O/trace.log; exit 1; }
python tools/profsum.py $O/trace 34 70 > $O/step_kernels.txt
head -45 $O/step_kernels.txt | cut -c1-200
tail -1 $O/step_kernels.txt
