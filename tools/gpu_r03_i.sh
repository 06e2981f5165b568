#!/bin/bash
# pack tiles + gated 4-row wgrad5: tests, timing, bench x2
set -o pipefail
O=gpurun_out/${TAG:-r03i}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_wgrad5.py tests/test_gpu_fusion_equivalence.py tests/test_gpu_ops.py tests/test_gpu_parity.py -k "wgrad or act_out or fused or pack or parity or golden or unet or attention" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
timeout -k 10 200 python -u tools/layerprof.py > $O/layerprof.txt 2>&1 || { echo "layerprof failed"; tail -20 $O/layerprof.txt; exit 1; }
grep -E "wgrad .*512x512|unet_pack_weights|unet_conv_wgrad" $O/layerprof.txt | cut -c1-120
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-line --no-graph-line > $O/bench_$k.json 2> $O/bench_$k.err || { echo "bench failed"; tail -20 $O/bench_$k.err; exit 1; }
  python -c "import json,sys; [print(f, json.load(open(f))['value']) for f in sys.argv[1:]]" $O/bench_$k.json
done
echo done
