#!/bin/bash
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/probe}
mkdir -p "$OUT"
: > "$OUT/probe.jsonl"
for p in ${PROBES:-0 8 15 7}; do
  CLONOS_DECODE=onepass CLONOS_ONE_PROBE=$p timeout -k 10 120 python3 tools/probe_one.py >> "$OUT/probe.jsonl" 2> "$OUT/probe_$p.err" || exit 1
done
CLONOS_DECODE=threepass timeout -k 10 120 python3 tools/probe_one.py >> "$OUT/probe.jsonl" 2> "$OUT/three.err" || exit 1
