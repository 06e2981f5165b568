#!/bin/bash
# conv5 correctness + per-layer timing (conv5 vs conv3), bench A/B, config/eval/graphed tests, full suite
set -o pipefail
O=gpurun_out/${TAG:-r03c}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv4.py tests/test_gpu_ops.py -k "conv4 or bn_backward_sums" -m gpu -q --timeout 300 --timeout-method thread > $O/conv_tests.log 2>&1
tail -25 $O/conv_tests.log
timeout -k 10 300 python -u tools/layerprof.py > $O/layerprof_c5.txt 2>&1 || { echo "layerprof failed"; tail -20 $O/layerprof_c5.txt; exit 1; }
UNET_CONV5=0 timeout -k 10 300 python -u tools/layerprof.py > $O/layerprof_c3.txt 2>&1 || { echo "layerprof c3 failed"; tail -20 $O/layerprof_c3.txt; exit 1; }
grep -E "conv5|conv3_kernel" $O/layerprof_c5.txt | head -40
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
UNET_CONV5=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line > $O/bench_c3.json 2> $O/bench_c3.err || { echo "bench c3 failed"; tail -20 $O/bench_c3.err; exit 1; }
cut -c1-400 $O/bench_c3.json
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_metrics.py tests/test_gpu_graphed.py -m gpu -v -s --timeout 300 --timeout-method thread > $O/cfg_tests.log 2>&1
grep -E "passed|failed|PASSED|FAILED|rel-L2|max\|d\||reductions|GradScaler|worst|Error" $O/cfg_tests.log | tail -60
