#!/bin/bash
# Decode A/B on one MI355X: GPU tests (default = one-pass decode), then bench.py's
# config-2 + config-3 legs with the one-pass kernel and with the three-pass pipeline.
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/r2c}
TESTS=${TESTS:-1}
mkdir -p "$OUT"
if [ "$TESTS" = 1 ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > "$OUT/tests.log" 2>&1 || exit 1
fi
CLONOS_DECODE=onepass timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inflight --no-config4 > "$OUT/one.json" 2> "$OUT/one.err" &&
CLONOS_DECODE=threepass timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-inflight --no-config4 > "$OUT/three.json" 2> "$OUT/three.err"
