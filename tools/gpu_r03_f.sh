#!/bin/bash
# conv5 BNB / act_out changes: conv tests, wgrad5 + fusion tests, per-layer timing, bench x2
set -o pipefail
O=gpurun_out/${TAG:-r03f}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_conv4.py tests/test_gpu_wgrad5.py tests/test_gpu_fusion_equivalence.py tests/test_gpu_ops.py -k "conv4 or conv5 or wgrad5 or act_out or fused or bn_backward_sums or conv_fwd or conv_dgrad or bench_tiles" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
timeout -k 10 200 python -u tools/layerprof.py > $O/layerprof.txt 2>&1 || { echo "layerprof failed"; tail -20 $O/layerprof.txt; exit 1; }
grep -A12 "per entry point" $O/layerprof.txt
grep "conv y .*512x512" $O/layerprof.txt | cut -c1-110
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-line --no-graph-line > $O/bench_$k.json 2> $O/bench_$k.err || { echo "bench failed"; tail -20 $O/bench_$k.err; exit 1; }
  python -c "import json,sys; [print(f, json.load(open(f))['value']) for f in sys.argv[1:]]" $O/bench_$k.json
done
echo done
