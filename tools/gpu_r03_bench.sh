#!/bin/bash
# Bench line (default config, with the graphed-step field), rocprofv3 kernel stats of the bench command,
# per-layer timing.  Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
O=gpurun_out/${TAG:-r03bench}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32-line --no-graph-line > $O/trace.log 2>&1 || { echo "trace failed"; tail -20 $O/trace.log; exit 1; }
python tools/profsum.py $O/trace/*/ 34 70 > $O/step_kernels.txt 2>&1 || python tools/profsum.py $O/trace 34 70 > $O/step_kernels.txt 2>&1
tail -1 $O/step_kernels.txt
timeout -k 10 200 python -u tools/layerprof.py > $O/layerprof.txt 2>&1 || { echo "layerprof failed"; tail -20 $O/layerprof.txt; exit 1; }
tail -30 $O/layerprof.txt
echo done
