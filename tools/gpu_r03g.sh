#!/bin/bash
# A/B: default conv5 policy vs conv3 everywhere (same box, alternating), then the config / eval-mode tests
set -o pipefail
O=gpurun_out/${TAG:-r03g}
mkdir -p $O
export TMPDIR=/tmp
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-line > $O/bench_def_$k.json 2> $O/bench_def_$k.err || { echo "bench failed"; tail -20 $O/bench_def_$k.err; exit 1; }
  UNET_CONV5=0 timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-line > $O/bench_c3_$k.json 2> $O/bench_c3_$k.err || { echo "bench c3 failed"; tail -20 $O/bench_c3_$k.err; exit 1; }
  python -c "import json,sys; [print(f, json.load(open(f))['value']) for f in sys.argv[1:]]" $O/bench_def_$k.json $O/bench_c3_$k.json
done
timeout -k 10 1000 python -u -m pytest tests/test_gpu_configs.py -m gpu -v -s --timeout 400 --timeout-method thread > $O/cfg_tests.log 2>&1
grep -E "passed|failed|PASSED|FAILED|rel-L2|Error|first fused" $O/cfg_tests.log | cut -c1-250 | tail -50
