#!/bin/bash
# quick GPU check: op-level parity tests (+ optional model tests), bench line, per-launch timing
set -o pipefail
O=gpurun_out/${TAG:-quick}
mkdir -p $O
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_ops.py} -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 200 python -u tools/layerprof.py > $O/layerprof.txt 2>&1 || { echo "layerprof failed"; tail -20 $O/layerprof.txt; exit 1; }
tail -22 $O/layerprof.txt
