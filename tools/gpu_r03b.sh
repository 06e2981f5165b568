#!/bin/bash
# conv4 ablations, then the config / eval / BN-sums / graphed tests and the rest of the suite (conv4 off)
set -o pipefail
O=gpurun_out/${TAG:-r03b}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/conv4_ablate.py > $O/conv4_ablate.txt 2>&1 || { echo "ablate failed"; tail -20 $O/conv4_ablate.txt; exit 1; }
cat $O/conv4_ablate.txt
timeout -k 10 300 python -u tools/conv_ablate.py 0,1,2,3,8,11,15,100,102,200,202 > $O/conv3_ablate.txt 2>&1 || { echo "ablate3 failed"; tail -20 $O/conv3_ablate.txt; exit 1; }
cat $O/conv3_ablate.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_metrics.py tests/test_gpu_graphed.py -m gpu -v -s --timeout 300 --timeout-method thread > $O/cfg_tests.log 2>&1
grep -E "passed|failed|PASSED|FAILED|rel-L2|max\|d\||reductions|GradScaler|worst|Error" $O/cfg_tests.log | tail -60
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_configs.py --deselect tests/test_gpu_graphed.py --deselect tests/test_gpu_metrics.py > $O/gpu_tests.log 2>&1
tail -15 $O/gpu_tests.log
