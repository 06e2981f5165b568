#!/bin/bash
# wgrad5 stall breakdown (SQ counters) on two layer shapes; the graphed-step crash with a Python fault trace;
# bench A/B wgrad5 vs wgrad2 without the graph line
set -o pipefail
O=gpurun_out/${TAG:-r03w5pmc}; mkdir -p $O
export TMPDIR=/tmp
for shp in "4 512 512 64 64" "4 256 256 128 128"; do
  tag=$(echo $shp | tr ' ' x)
  i=0
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR"; do
    i=$((i+1))
    UNET_WGRAD5=1 timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex 'wgrad5_kernel' --output-format csv -d $O/p${tag}_$i -o pmc -- python tools/wgrad_one.py $shp 4 > $O/p${tag}_$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p${tag}_$i.log; exit 1; }
    python tools/pmcsum.py $O/p${tag}_$i wgrad5 2>/dev/null | cut -c1-400
  done
done
timeout -k 10 300 python -u -X faulthandler bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fp32-line > $O/bench_graph.json 2> $O/bench_graph.err
echo "graph bench rc=$?"; grep -v "^\s*$" $O/bench_graph.err | grep -v UserWarning | tail -25 | cut -c1-200
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-line --no-graph-line > $O/bench_def_$k.json 2> $O/bench_def_$k.err || { echo "bench failed"; tail -20 $O/bench_def_$k.err; exit 1; }
  UNET_WGRAD5=0 timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-line --no-graph-line > $O/bench_w2_$k.json 2> $O/bench_w2_$k.err || { echo "bench w2 failed"; tail -20 $O/bench_w2_$k.err; exit 1; }
  python -c "import json,sys; [print(f, json.load(open(f))['value']) for f in sys.argv[1:]]" $O/bench_def_$k.json $O/bench_w2_$k.json
done
echo done
