#!/bin/bash
set -o pipefail
O=gpurun_out/${TAG:-r03d}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/conv4_ablate.py 0,1,2,3,4,8,16,7,15,31 --conv5 > $O/conv5_ablate.txt 2>&1 || { echo "ablate failed"; tail -20 $O/conv5_ablate.txt; exit 1; }
cat $O/conv5_ablate.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -m gpu -v -s --timeout 300 --timeout-method thread > $O/cfg_tests.log 2>&1
grep -E "passed|failed|PASSED|FAILED|rel-L2|max\|d\||reductions|GradScaler|worst|Error|first fused" $O/cfg_tests.log | tail -60
