set -o pipefail
O=gpurun_out/w4; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --probe 'conv3_kernel<bf16,3,1,4,2,8,1>' > $O/b_w4.json 2>$O/e1 || exit 1
UNET_CONV3_TILE=16 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_16.json 2>$O/e2 || exit 1
timeout -k 10 200 python -u tools/layerprof.py > $O/lp_w4.txt 2>&1 || exit 1
UNET_CONV3_TILE=16 timeout -k 10 200 python -u tools/layerprof.py > $O/lp_16.txt 2>&1 || exit 1
head -c 300 $O/b_w4.json; echo; head -c 300 $O/b_16.json
