#!/bin/bash
# conv5 with inline-asm DMAs: correctness, ablations, per-layer timing, bench A/B
set -o pipefail
O=gpurun_out/${TAG:-r03e}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv4.py tests/test_gpu_ops.py -k "conv4 or bn_backward_sums" -m gpu -q --timeout 300 --timeout-method thread > $O/conv_tests.log 2>&1
tail -5 $O/conv_tests.log
grep -q " passed" $O/conv_tests.log && ! grep -q "failed" $O/conv_tests.log || { echo "conv tests failed"; grep -E "FAILED|Error" $O/conv_tests.log | head; exit 1; }
timeout -k 10 300 python -u tools/conv4_ablate.py 0,1,2,4,8,16,31 --conv5 > $O/conv5_ablate.txt 2>&1 || { echo "ablate failed"; tail -20 $O/conv5_ablate.txt; exit 1; }
cat $O/conv5_ablate.txt
timeout -k 10 300 python -u tools/layerprof.py > $O/layerprof_c5.txt 2>&1 || { echo "layerprof failed"; tail -20 $O/layerprof_c5.txt; exit 1; }
grep -E "conv5|conv3_kernel" $O/layerprof_c5.txt | head -40
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
