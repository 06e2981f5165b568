#!/bin/bash
# GPU evidence steps, one parameterised script.
#   TAG=<dir under gpurun_out>  STEPS="tests smoke bench c5 c2 trace layerprof pmc sq ablate ab lp gdiag repro"  bash tools/gpu_steps.sh
# Every GPU step runs under its own time limit; the chain stops at the first failure (no retries).
set -o pipefail
O=gpurun_out/${TAG:-run}
mkdir -p $O
export TMPDIR=/tmp
fail() { echo "$1 failed"; tail -${3:-30} "$2"; exit 1; }
for step in ${STEPS:-tests smoke bench}; do
  case $step in
  tests)   # the driver's -m gpu suite, with per-test durations
    timeout -k 10 ${TLIM:-1100} python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread --durations=40 ${PYARGS} > $O/gpu_tests.log 2>&1 \
      || { grep -E "FAILED|Error|passed|failed" $O/gpu_tests.log | tail -20; fail tests $O/gpu_tests.log 60; }
    grep -E "passed|failed" $O/gpu_tests.log | tail -2 ;;
  some)    # a subset: PYARGS selects
    env ${PYENV} timeout -k 10 ${TLIM:-900} python -u -m pytest -m gpu -x -v --timeout 400 --timeout-method thread --durations=20 ${PYARGS} ${PYK:+-k "$PYK"} > $O/some_tests.log 2>&1 \
      || fail some $O/some_tests.log 60
    grep -E "passed|failed" $O/some_tests.log | tail -2 ;;
  smoke)
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || fail smoke $O/smoke.log
    tail -1 $O/smoke.log ;;
  bench)   # the driver's default bench line
    timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || fail bench $O/bench.err
    cat $O/bench.json ;;
  benchq)  # a quick headline-only line
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-fp32-line --no-graph-line ${BARGS} > $O/benchq.json 2> $O/benchq.err || fail benchq $O/benchq.err
    cat $O/benchq.json ;;
  c5)
    timeout -k 10 300 python -u bench.py --precision fp16 --in-ch 3 --size 1024 --accum 8 --steps 5 --warmup 2 --no-cpu-baseline --no-fp32-line > $O/bench_c5.json 2> $O/bench_c5.err || fail c5 $O/bench_c5.err
    cat $O/bench_c5.json ;;
  c2)
    timeout -k 10 300 python -u bench.py --model unet --no-cpu-baseline --no-fp32-line --no-graph-line > $O/bench_c2.json 2> $O/bench_c2.err || fail c2 $O/bench_c2.err
    cat $O/bench_c2.json ;;
  trace)   # kernel-trace stats of the bench command
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-line --no-graph-line > $O/trace.log 2>&1 || fail trace $O/trace.log
    # 78 traced steps: 5 warm-up + 30 timed + 10 probe + 2 hbm-probe + 31 fwd+bwd-only (without_optimizer)
    python tools/profsum.py $O/trace 78 45 "conv5_kernelIDF16b|conv5w_kernelIDF16b|conv3_kernelIDF16bLi3E|unet::conv5_kernel<" "conv5_splitk_finish_kernel" > $O/trace_summary.txt 2>&1; tail -3 $O/trace_summary.txt ;;
  layerprof)
    timeout -k 10 300 python -u tools/layerprof.py > $O/layerprof.txt 2>&1 || fail layerprof $O/layerprof.txt
    tail -5 $O/layerprof.txt ;;
  pmc)     # HBM bytes of the conv family and of the HBM-bound kernels (FETCH_SIZE and WRITE_SIZE in separate passes)
    i=0
    for set in FETCH_SIZE WRITE_SIZE; do
      i=$((i+1))
      timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/pmc$i -o pmc -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fp32-line --no-graph-line > $O/pmc$i.log 2>&1 || fail "pmc pass $i" $O/pmc$i.log 5
    done
    python tools/traffic.py --all $O/pmc1 $O/pmc2 > $O/traffic.log 2>&1 || fail traffic $O/traffic.log
    cp profiles/traffic.json $O/traffic.json
    tail -40 $O/traffic.log ;;
  pmc5)    # the same two passes over the C5 workload (fp16 3x1024^2, one micro-step per step): traffic.json "@1024x3" keys
    i=0
    for set in FETCH_SIZE WRITE_SIZE; do
      i=$((i+1))
      timeout -s KILL 180 rocprofv3 --pmc $set --output-format csv -d $O/pmc5_$i -o pmc -- python bench.py --precision fp16 --in-ch 3 --size 1024 --steps 1 --warmup 1 --no-cpu-baseline --no-fp32-line --no-graph-line > $O/pmc5_$i.log 2>&1 || fail "pmc5 pass $i" $O/pmc5_$i.log 5
    done
    python tools/traffic.py --all $O/pmc5_1 $O/pmc5_2 @1024x3 > $O/traffic5.log 2>&1 || fail traffic5 $O/traffic5.log
    cp profiles/traffic.json $O/traffic.json
    grep "@1024x3" $O/traffic5.log | head -20 ;;
  sq)      # instruction mix of the conv5 / wgrad5 kernels (SQ counters, one pass)
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_BRANCH --kernel-include-regex "${SQRE:-conv5_kernel|wgrad5_kernel}" --output-format csv -d $O/sq -o sq -- python tools/layerprof.py > $O/sq.log 2>&1 || fail sq $O/sq.log 5
    python tools/pmcsum.py $O/sq "${SQRE:-conv5_kernel|wgrad5_kernel}" > $O/sq_summary.txt 2>&1; cat $O/sq_summary.txt | head -40 ;;
  ablate)
    timeout -k 10 300 python -u tools/conv5_ablate.py ${ABL:-0,4,16,31} > $O/conv5_ablate.txt 2>&1 || fail ablate $O/conv5_ablate.txt
    cat $O/conv5_ablate.txt ;;
  ab)      # A/B(/C) of environment switches on one box: layer timing + the quick bench line, A B (C) A
    for v in "${ABA:-}" "${ABB:-}" ${ABC:+"$ABC"}; do
      env $v timeout -k 10 300 python -u tools/layerprof.py > "$O/layerprof_${v//[^A-Za-z0-9]/_}.txt" 2>&1 || fail "ab layerprof $v" "$O/layerprof_${v//[^A-Za-z0-9]/_}.txt"
    done
    for v in "${ABA:-}" "${ABB:-}" ${ABC:+"$ABC"} "${ABA:-}"; do
      env $v timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-line --no-graph-line > $O/ab.json 2> $O/ab.err || fail "ab bench $v" $O/ab.err
      echo "[$v] $(python -c "import json;d=json.load(open('$O/ab.json'));print(d['value'],d['ms_per_step'],d['roofline']['avg_us'])")"
    done ;;
  lp)      # layer timing under several environment settings (LPS: ';'-separated), summary lines matching LPGREP
    IFS=';' read -ra cfgs <<< "${LPS:-}"
    for v in "${cfgs[@]}"; do
      f="$O/lp_${v//[^A-Za-z0-9]/_}.txt"
      env $v timeout -k 10 300 python -u tools/layerprof.py > "$f" 2>&1 || fail "lp $v" "$f"
      echo "[$v]"; grep -E "${LPGREP:-total}" "$f" | head -${LPN:-20}
    done ;;
  guard)   # bounds-checked sweep (UNET_GUARD=1: guard bands around every allocation, checked after every library call)
    UNET_GUARD=1 timeout -k 10 ${TLIM:-900} python -u tools/guard_sweep.py ${GUARDARGS} > $O/guard.log 2>&1 || fail guard $O/guard.log 40
    grep -v amdgpu.ids $O/guard.log | tail -25 ;;
  faulttrace)  # the round-4 fault test once, bounds-checked (UNET_GUARD=1: our and torch's allocations) under a kernel trace
    UNET_GUARD=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ft -o ft -- python -u -m pytest -x -v -s -p no:cacheprovider tests/test_gpu_parity.py::test_fp16_grad_scaler_steps > $O/faulttrace.log 2>&1 || fail faulttrace $O/faulttrace.log 40
    find $O/ft -name "*kernel_trace.csv" -delete   # keep the stats (the per-dispatch trace of a guarded run is > 64 MiB)
    grep -E "passed|failed|Guard" $O/faulttrace.log | tail -3 ;;
  gdiag)
    timeout -k 10 180 python -u tools/graphed_diag.py > $O/graphed_diag.log 2>&1 || fail gdiag $O/graphed_diag.log 40
    cat $O/graphed_diag.log | grep -v amdgpu.ids ;;
  repro)   # round 3's GraphedTrainStep crash (old capture path); last in a call: it may end in a segfault
    PYTHONFAULTHANDLER=1 timeout -k 10 180 python -u tools/repro_graphed_live_graph.py ${REPRO:-backward} > $O/repro.log 2>&1; echo "repro rc $?" >> $O/repro.log
    tail -40 $O/repro.log ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo done
