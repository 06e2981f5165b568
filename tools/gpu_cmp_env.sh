#!/bin/bash
# A/B of an environment switch: op tests with it on, then bench + per-launch profile off and on.
# usage: VAR=NAME VAL=value bash tools/gpu_cmp_env.sh
set -o pipefail
O=gpurun_out/cmp_$VAR; mkdir -p $O
env $VAR=$VAL timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_off.json 2>$O/e1 || exit 1
env $VAR=$VAL timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_on.json 2>$O/e2 || exit 1
timeout -k 10 200 python -u tools/layerprof.py > $O/lp_off.txt 2>&1 || exit 1
env $VAR=$VAL timeout -k 10 200 python -u tools/layerprof.py > $O/lp_on.txt 2>&1 || exit 1
head -c 200 $O/b_off.json; echo; head -c 200 $O/b_on.json
