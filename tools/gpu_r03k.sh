#!/bin/bash
# conv5 (scalar-light loop): correctness, ablations, SALU/VALU counters, bench A/B vs conv3
set -o pipefail
O=gpurun_out/${TAG:-r03k}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv4.py tests/test_gpu_ops.py -k "conv4 or bn_backward_sums" -m gpu -q --timeout 300 --timeout-method thread > $O/conv_tests.log 2>&1
tail -3 $O/conv_tests.log
grep -q " passed" $O/conv_tests.log && ! grep -q "failed\|error" $O/conv_tests.log || { echo "conv tests failed"; grep -E "FAILED|Error" $O/conv_tests.log | head; exit 1; }
timeout -k 10 300 python -u tools/conv4_ablate.py 0,1,4,8,16,31 --conv5 > $O/conv5_ablate.txt 2>&1 || { echo "ablate failed"; tail -20 $O/conv5_ablate.txt; exit 1; }
cat $O/conv5_ablate.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_BRANCH --kernel-include-regex "conv5_kernel" --output-format csv -d $O/p1 -o pmc -- python tools/conv4_ablate.py 0,31 --conv5 > $O/p1.log 2>&1 || { echo "pmc failed"; tail -5 $O/p1.log; exit 1; }
python tools/pmcsum.py $O/p1 conv5_kernel | cut -c1-300
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-line > $O/bench_def_$k.json 2> $O/bench_def_$k.err || { echo "bench failed"; tail -20 $O/bench_def_$k.err; exit 1; }
  UNET_CONV5=0 timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-line > $O/bench_c3_$k.json 2> $O/bench_c3_$k.err || { echo "bench c3 failed"; tail -20 $O/bench_c3_$k.err; exit 1; }
  python -c "import json,sys; [print(f, json.load(open(f))['value']) for f in sys.argv[1:]]" $O/bench_def_$k.json $O/bench_c3_$k.json
done
UNET_CONV5=1 timeout -k 10 300 python -u tools/layerprof.py > $O/layerprof_c5.txt 2>&1 || { echo "layerprof failed"; tail -20 $O/layerprof_c5.txt; exit 1; }
grep -E "conv5|conv3_kernel" $O/layerprof_c5.txt | cut -c1-120 | head -40
