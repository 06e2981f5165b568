#!/bin/bash
# F32 counted-store epilogue + one-launch slab reduce: op tests, per-layer timing (default / conv5 everywhere), bench x2
set -o pipefail
O=gpurun_out/${TAG:-r03h}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_conv4.py tests/test_gpu_wgrad5.py tests/test_gpu_fusion_equivalence.py tests/test_gpu_ops.py -k "conv4 or conv5 or wgrad or act_out or fused or bn_backward_sums or conv_fwd or conv_dgrad or bench_tiles or pw_" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
for w in 1 0; do WG_KIND=act UNET_WGRAD5=$w timeout -k 10 60 python tools/wgrad_one.py 4 512 512 64 64 20 > $O/one.log 2>&1 || { tail -5 $O/one.log; exit 1; }; tail -1 $O/one.log; done
timeout -k 10 200 python -u tools/layerprof.py > $O/layerprof.txt 2>&1 || { echo "layerprof failed"; tail -20 $O/layerprof.txt; exit 1; }
UNET_CONV5=1 timeout -k 10 200 python -u tools/layerprof.py > $O/layerprof_c5.txt 2>&1 || { echo "layerprof failed"; tail -20 $O/layerprof_c5.txt; exit 1; }
grep -A8 "per entry point" $O/layerprof.txt
paste <(grep "conv f32" $O/layerprof.txt | cut -c1-112) <(grep "conv f32" $O/layerprof_c5.txt | cut -c1-12)
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-line --no-graph-line > $O/bench_$k.json 2> $O/bench_$k.err || { echo "bench failed"; tail -20 $O/bench_$k.err; exit 1; }
  python -c "import json,sys; [print(f, json.load(open(f))['value']) for f in sys.argv[1:]]" $O/bench_$k.json
done
echo done
