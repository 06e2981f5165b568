#!/bin/bash
# new-path tests (wgrad5, act_out, outconv+BN fusion, smallcin MFMA), wgrad timing table, bench
set -o pipefail
O=gpurun_out/${TAG:-r03c}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_wgrad5.py tests/test_gpu_fusion_equivalence.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
for shp in "4 512 512 64 64" "4 256 256 64 128" "4 256 256 128 128" "4 128 128 256 256" "4 64 64 512 512"; do
  for k in plain act; do
    for w in 1 0; do
      WG_KIND=$k UNET_WGRAD5=$w timeout -k 10 60 python tools/wgrad_one.py $shp 20 > $O/one.log 2>&1 || { tail -5 $O/one.log; exit 1; }
      tail -1 $O/one.log
    done
  done
done | tee $O/wtime.txt
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-line --no-graph-line > $O/bench_def_$k.json 2> $O/bench_def_$k.err || { echo "bench failed"; tail -20 $O/bench_def_$k.err; exit 1; }
  UNET_WGRAD5=0 timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-line --no-graph-line > $O/bench_w2_$k.json 2> $O/bench_w2_$k.err || { echo "bench w2 failed"; tail -20 $O/bench_w2_$k.err; exit 1; }
  python -c "import json,sys; [print(f, json.load(open(f))['value']) for f in sys.argv[1:]]" $O/bench_def_$k.json $O/bench_w2_$k.json
done
echo done
