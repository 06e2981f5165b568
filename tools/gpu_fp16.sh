#!/bin/bash
# fp16 operand mode on one GPU: op / model / GradScaler tests, then bench lines (C3 bf16, C3 fp16, C5 fp16).
set -o pipefail
O=gpurun_out/${TAG:-f16}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_parity.py \
  -k "fp16 or 16bit or scaler" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line > $O/bench_bf16.json 2> $O/bench_bf16.err || { tail -20 $O/bench_bf16.err; exit 1; }
cat $O/bench_bf16.json
timeout -k 10 300 python -u bench.py --precision fp16 --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line > $O/bench_fp16.json 2> $O/bench_fp16.err || { tail -20 $O/bench_fp16.err; exit 1; }
cat $O/bench_fp16.json
timeout -k 10 400 python -u bench.py --precision fp16 --in-ch 3 --size 1024 --accum 8 --steps 3 --warmup 2 --no-cpu-baseline --no-fp32-line > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
cat $O/bench_c5.json
