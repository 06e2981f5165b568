#!/bin/bash
# A/B of host-side switches on one box: bench.py (no CPU baseline / fp32 line) under each env setting in
# turn, twice, so box-to-box variance does not enter the comparison.  usage: AB="VAR1=1|VAR2=1" tools/gpu_ab.sh
set -o pipefail
O=gpurun_out/${TAG:-ab}
mkdir -p $O
IFS='|' read -ra SETS <<< "${AB:-}"
for rep in 1 2; do
  for s in "" "${SETS[@]}"; do
    env $s timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line > $O/b.json 2> $O/b.err || { echo "bench failed ($s)"; tail -5 $O/b.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/b.json')); print('rep $rep [${s:-default}]', d['value'], d['ms_per_step'], d['without_optimizer']['value'])"
  done
done
