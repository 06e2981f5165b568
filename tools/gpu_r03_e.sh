#!/bin/bash
# wgrad5 tests + plain-source timing (TH=4 stages for 64-channel blocks), then per-layer timing / trace (r03_d)
set -o pipefail
O=gpurun_out/${TAG:-r03e}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_wgrad5.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
for shp in "4 512 512 64 64" "4 256 256 128 64" "4 512 512 128 64"; do
  for w in 1 0; do
    WG_KIND=plain UNET_WGRAD5=$w timeout -k 10 60 python tools/wgrad_one.py $shp 20 > $O/one.log 2>&1 || { tail -5 $O/one.log; exit 1; }
    tail -1 $O/one.log
  done
done | tee $O/wtime.txt
TAG=$TAG tools/gpu_r03_d.sh
