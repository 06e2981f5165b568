set -o pipefail
O=gpurun_out/fp16pw; mkdir -p $O
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_gpu_ops.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_fusion_equivalence.py} -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 300 python -u bench.py --precision fp16 --in-ch 3 --size 1024 --accum 8 --steps 2 --warmup 1 --no-cpu-baseline --no-fp32-line > $O/c5.json 2> $O/c5.err || { tail -5 $O/c5.err; exit 1; }
cat $O/c5.json
timeout -k 10 200 python -u tools/layerprof.py --prec fp16 --size 1024 --batch 4 > $O/lp.txt 2>&1 || { tail -5 $O/lp.txt; exit 1; }
