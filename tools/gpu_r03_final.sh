#!/bin/bash
# Final round-3 check on the final tree: the full -m gpu suite + smoke (tools/gpu_tests_only.sh), then the
# default bench line and the kernel-trace stats of the bench command.
set -o pipefail
export TAG=${TAG:-r03final}
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_tests_only.sh || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32-line --no-graph-line > $O/trace.log 2>&1 || { echo "trace failed"; tail -20 $O/trace.log; exit 1; }
echo done
