#!/bin/bash
# Round profile on one MI355X (run under gpurun from the repo root):
#   1. bench.py (full config, CPU baseline included)          -> $OUT/bench.json
#   2. rocprofv3 --kernel-trace --stats over bench.py          -> $OUT/trace/
#   3. separate PMC passes FETCH_SIZE / WRITE_SIZE (kernel trace only, no sys/runtime trace)
#   4. rocprofv3 --kernel-trace --stats over the in-flight replay leg alone  -> $OUT/ifl_trace/
# Every GPU step has its own time limit and the steps are chained with &&.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/round}
mkdir -p "$OUT"
timeout -k 10 420 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-config3 --no-inflight --no-isolated > "$OUT/trace.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config3 --no-inflight --no-isolated > "$OUT/fetch.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config3 --no-inflight --no-isolated > "$OUT/write.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/ifl_trace" -o run --output-format csv -- \
    python3 bench.py --inflight-only --no-cpu-baseline > "$OUT/ifl_trace.log" 2>&1
