#!/bin/bash
# per-layer timing with / without the BN-backward-sums dgrad epilogue; kernel trace of the bench step
set -o pipefail
O=gpurun_out/${TAG:-r03d}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/layerprof.py > $O/layerprof.txt 2>&1 || { echo "layerprof failed"; tail -20 $O/layerprof.txt; exit 1; }
UNET_NO_BNB_FUSE=1 timeout -k 10 200 python -u tools/layerprof.py > $O/layerprof_nobnb.txt 2>&1 || { echo "layerprof failed"; tail -20 $O/layerprof_nobnb.txt; exit 1; }
grep -A40 "per entry point" $O/layerprof.txt | head -30
grep -A40 "per entry point" $O/layerprof_nobnb.txt | head -30
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32-line --no-graph-line > $O/trace.log 2>&1 || { echo "trace failed"; tail -20 $O/trace.log; exit 1; }
python tools/profsum.py $(dirname $(ls $O/trace/*/*kernel_stats.csv 2>/dev/null || ls $O/trace/*kernel_stats.csv)) 34 70 > $O/step_kernels.txt 2>&1
cat $O/step_kernels.txt | cut -c1-150
echo done
