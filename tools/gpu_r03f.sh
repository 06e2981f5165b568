#!/bin/bash
set -o pipefail
O=gpurun_out/r03f
mkdir -p $O
export TMPDIR=/tmp
UNET_CONV5_DBG=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_conv4.py -k "conv5 and act_gate" -m gpu -q --timeout 120 --timeout-method thread > $O/dbg1.log 2>&1
tail -3 $O/dbg1.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv4.py -k "conv5 and act_gate" -m gpu -q --timeout 120 --timeout-method thread > $O/dbg0.log 2>&1
tail -3 $O/dbg0.log
exit 0
