#!/bin/bash
# GPU call: config 4/5 scatter with the candidate scan after the copy (default) and before it
# (ab/libsidefirst.so), twice each
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/abs; rm -rf $O; mkdir -p $O
for v in base first base first; do
  if [ $v = first ]; then export CLONOS_LIB=$PWD/ab/libsidefirst.so; else unset CLONOS_LIB; fi
  timeout -k 10 200 python3 bench.py --config4-only > $O/$v.json 2> $O/$v.err || exit 3
  python3 - "$O/$v.json" $v <<'P'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c4, c5 = d["config4"], d["config5"]
print(sys.argv[2], "c4", c4["ms_per_step"], c4["kernels_rank0"]["upstream_scatter"]["avg_ms"], "c5", c5["latency_ms"],
      c5["kernels_rank0"]["upstream_scatter"]["avg_ms"])
P
done
