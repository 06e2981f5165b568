#!/bin/bash
# wgrad5: op tests (both paths vs torch), per-layer timing with wgrad5 on / off, bench A/B
set -o pipefail
O=gpurun_out/${TAG:-r03w5}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_wgrad5.py tests/test_gpu_ops.py -k "wgrad or first_conv" -x -q --timeout 120 --timeout-method thread > $O/w5_tests.log 2>&1
rc=$?
tail -5 $O/w5_tests.log
[ $rc -eq 0 ] || { echo "wgrad5 tests failed rc=$rc"; grep -E "FAILED|Error|assert" $O/w5_tests.log | head -20; exit 1; }
UNET_WGRAD5=1 timeout -k 10 200 python -u tools/layerprof.py > $O/layerprof_w5.txt 2>&1 || { echo "layerprof failed"; tail -20 $O/layerprof_w5.txt; exit 1; }
UNET_WGRAD5=0 timeout -k 10 200 python -u tools/layerprof.py > $O/layerprof_w2.txt 2>&1 || { echo "layerprof failed"; tail -20 $O/layerprof_w2.txt; exit 1; }
paste <(grep wgrad $O/layerprof_w5.txt | cut -c1-110) <(grep wgrad $O/layerprof_w2.txt | cut -c1-24)
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-line > $O/bench_def_$k.json 2> $O/bench_def_$k.err || { echo "bench failed"; tail -20 $O/bench_def_$k.err; exit 1; }
  UNET_WGRAD5=0 timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-line --no-graph-line > $O/bench_w2_$k.json 2> $O/bench_w2_$k.err || { echo "bench w2 failed"; tail -20 $O/bench_w2_$k.err; exit 1; }
  python -c "import json,sys; [print(f, json.load(open(f))['value'], json.load(open(f)).get('graphed_step')) for f in sys.argv[1:]]" $O/bench_def_$k.json $O/bench_w2_$k.json
done
echo done
