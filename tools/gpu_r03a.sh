#!/bin/bash
# round-3 GPU check: conv4 op tests, per-layer timing conv4 vs conv3, the new config / eval-mode / BN-sums
# tests, the rest of the GPU suite, bench lines with and without conv4
set -o pipefail
O=gpurun_out/${TAG:-r03a}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv4.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/conv4_tests.log 2>&1 || { echo "conv4 tests failed"; tail -60 $O/conv4_tests.log; exit 1; }
tail -2 $O/conv4_tests.log
timeout -k 10 300 python -u tools/layerprof.py > $O/layerprof_c4.txt 2>&1 || { echo "layerprof failed"; tail -20 $O/layerprof_c4.txt; exit 1; }
UNET_CONV4=0 timeout -k 10 300 python -u tools/layerprof.py > $O/layerprof_c3.txt 2>&1 || { echo "layerprof c3 failed"; tail -20 $O/layerprof_c3.txt; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
UNET_CONV4=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line > $O/bench_c3.json 2> $O/bench_c3.err || { echo "bench c3 failed"; tail -20 $O/bench_c3.err; exit 1; }
cat $O/bench_c3.json
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_metrics.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/cfg_tests.log 2>&1 || { echo "config tests failed"; tail -60 $O/cfg_tests.log; exit 1; }
grep -E "passed|failed|rel-L2|max\|d\||reductions|GradScaler|worst" $O/cfg_tests.log | tail -40
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_configs.py --deselect tests/test_gpu_conv4.py > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
