#!/bin/bash
# The full -m gpu suite (as the driver runs it) plus smoke(), each under its own time limit.
set -o pipefail
O=gpurun_out/${TAG:-tests}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 ${TLIM:-1000} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=30 > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error|passed|failed" $O/gpu_tests.log | tail -20; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
echo done
