#!/bin/bash
# Round evidence: parity tests, the bench line (default + C5 variant), kernel-trace stats of the bench
# command, per-launch layer timing and the HBM-traffic PMC passes for the probed conv kernel.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
O=gpurun_out/${TAG:-round}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python -u bench.py --precision fp16 --in-ch 3 --size 1024 --accum 8 --steps 2 --warmup 1 --no-cpu-baseline --no-fp32-line > $O/bench_c5.json 2> $O/bench_c5.err || { echo "c5 bench failed"; tail -20 $O/bench_c5.err; exit 1; }
cat $O/bench_c5.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32-line > $O/trace.log 2>&1 || { echo "trace failed"; tail -20 $O/trace.log; exit 1; }
timeout -k 10 200 python -u tools/layerprof.py > $O/layerprof.txt 2>&1 || { echo "layerprof failed"; tail -20 $O/layerprof.txt; exit 1; }
i=0
for set in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex 'conv3_kernel' --output-format csv -d $O/pmc$i -o pmc -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fp32-line > $O/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pmc$i.log; exit 1; }
  python tools/pmcsum.py $O/pmc$i conv3_kernel
done
echo done
