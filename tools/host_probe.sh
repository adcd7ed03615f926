#!/bin/bash
# Host-side probe of the config-2 bench step: per-call host time (CLONOS_STEP_PROBE)
# and host phases inside the engine (CLONOS_HOST_PROF), plus a kernel trace of the same run.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/probe}
mkdir -p "$OUT"
C2="--steps 20 --warmup 3 --no-cpu-baseline --no-config3 --no-inflight --no-config4 --no-config1"
echo probe && CLONOS_STEP_PROBE=1 CLONOS_HOST_PROF=1 timeout -k 10 300 python -u bench.py $C2 > "$OUT/probe.json" 2> "$OUT/probe.err" &&
echo trace && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-config3 --no-inflight --no-isolated --no-config4 --no-config1 > "$OUT/trace.log" 2>&1 &&
echo done-c2 &&
echo c4 && CLONOS_HOST_PROF=1 timeout -k 10 300 python -u bench.py --config4-only --no-cpu-baseline > "$OUT/c4.json" 2> "$OUT/c4.err" &&
echo done-c4
