#!/bin/bash
# GPU call: config-2 step with the count grid's free blocks per CU at 0, 1 (default), 2; twice each
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/margin; rm -rf $O; mkdir -p $O
C2="--steps 20 --warmup 3 --no-cpu-baseline --no-config3 --no-inflight --no-isolated --no-config4 --no-config1"
for m in 1 0 2 1 0 2; do
  CLONOS_COUNT_MARGIN=$m timeout -k 10 200 python3 bench.py $C2 > $O/m$m.json 2> $O/m$m.err || exit 3
  python3 - $O/m$m.json $m <<'P'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print("margin", sys.argv[2], d["ms_per_step"], d["roofline"]["frac"])
P
done
