#!/bin/bash
# GPU check: the -m gpu suite (all failures listed), smoke, the default bench line.
# A test failure (pytest rc 1) still runs smoke and bench; a crash, abort or timeout stops.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/check}
mkdir -p "$OUT"
echo tests
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > "$OUT/gputest.log" 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
echo smoke && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
echo bench && timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" &&
echo done
