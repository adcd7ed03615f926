#!/bin/bash
# One GPU call, parameterised (replaces round 5's one-off tools/r5_*.sh scripts).  Run under
# gpurun from the repository root:
#   bash tools/gpu.sh STEP [STEP ...]
# Steps run in order, each under its own time limit; the first that fails (a test failure
# included) ends the call.  Output under $OUT (default gpurun_out/run).
#   tests[=files]      pytest -m gpu (all of tests/, or the comma-separated files)
#   smoke              __graft_entry__.smoke()
#   bench[=args]       bench.py (default arguments: the driver's default line)
#   c2[=N]             N config-2-only bench lines (default 3), $OUT/c2_<i>.json
#   trace              rocprofv3 --kernel-trace --stats of a short config-2 bench
#   pmc                tools/pmc.sh counter passes over the decode and gather kernels
#   fuzz[=minutes]     tests/fuzz_gpu_decode.py for that long (default 4)
#   rehearse[=N]       CLONOS_BENCH_REHEARSAL=1 bench at world N over gloo, all ranks on GPU 0
# Environment: BENCH_ENV (extra variables for bench steps, e.g. "CLONOS_GATHER_PRIO=0"),
# BENCH_ARGS (extra arguments for the rehearsal, e.g. "--logs 16 --records 200000").
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 2
OUT=${OUT:-gpurun_out/run}
mkdir -p "$OUT"
C2="--steps 20 --warmup 5 --no-cpu-baseline --no-config3 --no-inflight --no-config4 --no-config1"
run() {  # name, limit, command...
  local name=$1 lim=$2
  shift 2
  echo "== $name ($(date +%T))" >&2
  timeout -k 10 "$lim" "$@"
  local rc=$?
  echo "== $name rc=$rc" >&2
  return $rc
}
for step in "$@"; do
  key=${step%%=*}
  val=""
  [ "$key" != "$step" ] && val=${step#*=}
  case $key in
    tests)
      files=${val//,/ }
      run tests 1500 python -u -m pytest ${files:-tests} -m gpu -x -q --timeout 120 --timeout-method thread \
        > "$OUT/pytest.log" 2>&1
      rc=$?
      tail -5 "$OUT/pytest.log"
      [ $rc -eq 0 ] || exit $rc
      ;;
    smoke)
      run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
      tail -2 "$OUT/smoke.log"
      ;;
    bench)
      run bench 500 env $BENCH_ENV python3 bench.py $val > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
      cat "$OUT/bench.json"
      ;;
    c2)
      for i in $(seq 1 "${val:-3}"); do
        run "c2 $i" 200 env $BENCH_ENV python3 bench.py $C2 > "$OUT/c2_$i.json" 2> "$OUT/c2_$i.err" || exit $?
        python3 -c "import json,sys; d=json.load(open('$OUT/c2_$i.json')); print(d['ms_per_step'], d['roofline']['frac'])"
      done
      ;;
    trace)
      run trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
        python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-config3 --no-inflight --no-isolated \
        --no-config4 --no-config1 > "$OUT/trace.log" 2>&1 || exit $?
      python3 tools/timeline.py "$OUT/trace" 3 > "$OUT/timeline.txt" || exit 4
      ;;
    pmc)
      run pmc 900 bash tools/pmc.sh "$OUT/pmc" > "$OUT/pmc.log" 2>&1 || exit $?
      ;;
    fuzz)
      run fuzz $(( ${val:-4} * 60 + 120 )) python3 -u tests/fuzz_gpu_decode.py --minutes "${val:-4}" \
        > "$OUT/fuzz.log" 2>&1 || exit $?
      tail -3 "$OUT/fuzz.log"
      ;;
    rehearse)
      n=${val:-2}
      run "rehearse $n" 900 env CLONOS_BENCH_REHEARSAL=1 python3 bench.py --gpus "$n" --steps 5 --warmup 2 \
        --no-cpu-baseline $BENCH_ARGS > "$OUT/rehearse_w$n.json" 2> "$OUT/rehearse_w$n.err" || exit $?
      cat "$OUT/rehearse_w$n.json"
      ;;
    *)
      echo "unknown step $step"
      exit 2
      ;;
  esac
done
echo "== done"
