#!/bin/bash
# materialize_fast with 2 elements per trip: gate tests, then library A/B
set -o pipefail
O=gpurun_out/${TAG:-r03r}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_parity.py tests/test_gpu_fusion_equivalence.py tests/test_gpu_determinism.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-line --no-graph-line > $O/new_$k.json 2> $O/new_$k.err || { echo "bench failed"; tail -20 $O/new_$k.err; exit 1; }
  UNET_HIP_LIB=$PWD/tools/ab_old.so timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-line --no-graph-line > $O/old_$k.json 2> $O/old_$k.err || { echo "bench old failed"; tail -20 $O/old_$k.err; exit 1; }
  python -c "import json,sys; [print(f, json.load(open(f))['value'], json.load(open(f))['hbm']['kernels'].get('unet_materialize'), json.load(open(f))['hbm']['kernels'].get('unet_materialize_pool')) for f in sys.argv[1:]]" $O/new_$k.json $O/old_$k.json
done
echo done
