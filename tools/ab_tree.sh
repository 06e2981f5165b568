#!/bin/bash
# Same-box A/B of two whole trees: the working tree (B) against a copy of another commit's tree with its own built
# library under ab_<tag>/ (A; bench.py, the package, oracle/, tools/layerprof.py, profiles/traffic.json): the quick
# bench line A B A B and one layer profile each.  Every GPU step under its own time limit; stops at the first failure.
#   TAG=<out dir> AB=ab_r04 bash tools/ab_tree.sh
set -o pipefail
O=gpurun_out/${TAG:-ab}
A=${AB:-ab_r04}
mkdir -p $O
BARGS="--steps ${STEPS:-30} --warmup 5 --no-cpu-baseline --no-fp32-line --no-graph-line"
val() { python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['value'],d['ms_per_step'],d['roofline']['avg_us'])" "$1"; }
for r in 1 2; do
  (cd $A && timeout -k 10 300 python -u bench.py $BARGS) > $O/a$r.json 2> $O/a$r.err || { tail -20 $O/a$r.err; exit 1; }
  echo "A[$A] $(val $O/a$r.json)"
  timeout -k 10 300 python -u bench.py $BARGS > $O/b$r.json 2> $O/b$r.err || { tail -20 $O/b$r.err; exit 1; }
  echo "B[tree] $(val $O/b$r.json)"
done
(cd $A && timeout -k 10 300 python -u tools/layerprof.py) > $O/layerprof_a.txt 2>&1 || { tail -20 $O/layerprof_a.txt; exit 1; }
timeout -k 10 300 python -u tools/layerprof.py > $O/layerprof_b.txt 2>&1 || { tail -20 $O/layerprof_b.txt; exit 1; }
tail -n 3 "$O/layerprof_a.txt"; tail -n 3 "$O/layerprof_b.txt"
