#!/bin/bash
# PMC passes over tools/probe_one.py (config 2, 64 logs): instruction mix and waits of the
# decode kernels, one counter group per rocprofv3 pass (kernel trace only).
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/pmcp}
mkdir -p "$OUT"
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
G2="SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
i=0
for mode in "onepass:0" "onepass:7" "onepass:3" "threepass:0"; do
  dec=${mode%%:*}; pr=${mode##*:}
  for g in "$G1" "$G2"; do
    i=$((i+1))
    CLONOS_DECODE=$dec CLONOS_ONE_PROBE=$pr timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $g -d "$OUT/p$i" -o run --output-format csv -- python3 tools/probe_one.py 16 > "$OUT/p$i.log" 2>&1 || exit 1
    echo "p$i $dec $pr" >> "$OUT/index.txt"
  done
done
