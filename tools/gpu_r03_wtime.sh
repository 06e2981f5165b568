#!/bin/bash
# act_out + wgrad5 tests; wgrad timing: wgrad5 vs wgrad2, plain vs BN-activation source, the network's 3x3 shapes
set -o pipefail
O=gpurun_out/${TAG:-r03wtime}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_wgrad5.py tests/test_gpu_fusion_equivalence.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
for shp in "4 512 512 64 64" "4 256 256 64 128" "4 256 256 128 128" "4 128 128 256 256" "4 64 64 512 512" "4 32 32 512 512"; do
  for k in plain act; do
    for w in 1 0; do
      WG_KIND=$k UNET_WGRAD5=$w timeout -k 10 60 python tools/wgrad_one.py $shp 20 > $O/one.log 2>&1 || { tail -5 $O/one.log; exit 1; }
      tail -1 $O/one.log
    done
  done
done | tee $O/wtime.txt
echo done
