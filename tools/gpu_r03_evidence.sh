#!/bin/bash
# Round-3 evidence: HBM-traffic PMC passes for the probed conv family (C3 and C5, into profiles/traffic.json,
# which the bench lines then report), the default bench line, kernel-trace stats of the bench command,
# per-layer timing, the C5 line (fp16, 3x1024^2, accum 8) with its kernel stats, and the C2 (UNet) line.
set -o pipefail
O=gpurun_out/${TAG:-r03ev}; mkdir -p $O
export TMPDIR=/tmp
i=0
for set in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex 'conv[345]_kernel' --output-format csv -d $O/pmc$i -o pmc -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fp32-line --no-graph-line > $O/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pmc$i.log; exit 1; }
done
python tools/traffic.py $O/pmc1 $O/pmc2 "" "conv3_kernel<bf16,3,|conv4_kernel<bf16,|conv5_kernel<bf16,=conv3_kernel|conv4_kernel|conv5_kernel" > $O/traffic.log 2>&1 || { tail $O/traffic.log; exit 1; }
for set in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set --kernel-include-regex 'conv[345]_kernel' --output-format csv -d $O/pmc$i -o pmc -- python bench.py --precision fp16 --in-ch 3 --size 1024 --accum 8 --steps 1 --warmup 1 --no-cpu-baseline --no-fp32-line --no-graph-line > $O/pmc$i.log 2>&1 || { echo "c5 pmc pass $i failed"; tail -5 $O/pmc$i.log; exit 1; }
done
python tools/traffic.py $O/pmc3 $O/pmc4 "@1024x3" "conv3_kernel<fp16,3,|conv4_kernel<fp16,|conv5_kernel<fp16,=conv3_kernel|conv4_kernel|conv5_kernel" > $O/traffic_c5.log 2>&1 || { tail $O/traffic_c5.log; exit 1; }
cp profiles/traffic.json $O/traffic.json
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32-line --no-graph-line > $O/trace.log 2>&1 || { echo "trace failed"; tail -20 $O/trace.log; exit 1; }
timeout -k 10 200 python -u tools/layerprof.py > $O/layerprof.txt 2>&1 || { echo "layerprof failed"; tail -20 $O/layerprof.txt; exit 1; }
timeout -k 10 400 python -u bench.py --precision fp16 --in-ch 3 --size 1024 --accum 8 --steps 5 --warmup 2 --no-cpu-baseline --no-fp32-line > $O/bench_c5.json 2> $O/bench_c5.err || { echo "c5 bench failed"; tail -20 $O/bench_c5.err; exit 1; }
cut -c1-300 $O/bench_c5.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c5 -o run -- python bench.py --precision fp16 --in-ch 3 --size 1024 --accum 8 --steps 3 --warmup 1 --no-cpu-baseline --no-fp32-line > $O/trace_c5.log 2>&1 || { echo "c5 trace failed"; tail -20 $O/trace_c5.log; exit 1; }
timeout -k 10 400 python -u bench.py --model unet --no-cpu-baseline --no-fp32-line > $O/bench_c2.json 2> $O/bench_c2.err || { echo "c2 bench failed"; tail -20 $O/bench_c2.err; exit 1; }
cut -c1-300 $O/bench_c2.json
echo done
