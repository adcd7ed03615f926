#!/bin/bash
# GPU call: the config-2 step 12 times, abort reasons and redos per run (a rare slow run had one)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/redo; rm -rf $O; mkdir -p $O
C2="--steps 20 --warmup 3 --no-cpu-baseline --no-config3 --no-inflight --no-isolated --no-config4 --no-config1"
if [ -n "$PHASES" ]; then export CLONOS_SCAN_PHASES=/tmp/sp.bin; fi  # (the ex writers in the give-up dump)
for i in $(seq 1 ${RUNS:-12}); do
  CLONOS_FUSED_DEBUG=1 timeout -k 10 200 python3 bench.py $C2 > $O/r$i.json 2> $O/r$i.err || exit 3
  python3 - $O/r$i.json $i <<'P'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
k = {n: v["launches"] for n, v in d["kernels"].items() if n.startswith("decode_abort") or n.startswith("decode_async") or n == "decode_count"}
print(sys.argv[2], d["ms_per_step"], k)
P
  grep -h -e aborted -e "repair walk" -e "ex writer" -e "not taken" $O/r$i.err | head -24 || true
done
