#!/bin/bash
# A/B on one box: the in-tree library vs tools/ab_old.so (UNET_HIP_LIB), alternating, 3 rounds
set -o pipefail
O=gpurun_out/${TAG:-abl}; mkdir -p $O
export TMPDIR=/tmp
for k in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-line --no-graph-line > $O/new_$k.json 2> $O/new_$k.err || { echo "bench failed"; tail -20 $O/new_$k.err; exit 1; }
  UNET_HIP_LIB=$PWD/tools/ab_old.so timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-line --no-graph-line > $O/old_$k.json 2> $O/old_$k.err || { echo "bench old failed"; tail -20 $O/old_$k.err; exit 1; }
  python -c "import json,sys; [print(f, json.load(open(f))['value']) for f in sys.argv[1:]]" $O/new_$k.json $O/old_$k.json
done
echo done
