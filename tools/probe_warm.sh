#!/bin/bash
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/warm}
mkdir -p "$OUT"
: > "$OUT/probe.jsonl"
for w in 96 64 48 32 16; do
  CLONOS_DECODE=threepass CLONOS_WARM=$w timeout -k 10 120 python3 tools/probe_one.py >> "$OUT/probe.jsonl" 2> "$OUT/w$w.err" || exit 1
done
CLONOS_DECODE=threepass timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d "$OUT/pmc" -o run --output-format csv -- python3 tools/probe_one.py 16 > "$OUT/pmc.log" 2>&1
