#!/bin/bash
# Round-5 check: the -m gpu suite, then config-2 bench A/B (decodes in flight x stream
# priority mode) and kernel traces for tools/timeline.py.  A test failure (rc 1) still runs
# the benches; a crash, abort or timeout stops.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/r5check}; rm -rf $OUT; mkdir -p $OUT
echo tests
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread ${TESTS:-} > $OUT/gputest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 $OUT/gputest.log
[ $rc -le 1 ] || exit $rc
C2="--steps 20 --warmup 5 --no-cpu-baseline --no-config3 --no-inflight --no-config4 --no-config1"
for v in "1 1" "1 0" "1 2" "0 1" "0 2"; do
  set -- $v
  echo "bench pipeline=$1 prio=$2"
  CLONOS_BENCH_PIPELINE=$1 CLONOS_GATHER_PRIO=$2 timeout -k 10 200 python3 bench.py $C2 > $OUT/b_$1$2.json 2> $OUT/b_$1$2.err || exit 3
done
for pr in 1 2; do
  echo trace $pr && CLONOS_GATHER_PRIO=$pr timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace$pr -o run --output-format csv -- \
      python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-config3 --no-inflight --no-isolated --no-config4 --no-config1 > $OUT/trace$pr.log 2>&1 &&
  python3 tools/timeline.py $OUT/trace$pr 3 > $OUT/timeline$pr.txt || exit 4
done
echo done
