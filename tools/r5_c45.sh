#!/bin/bash
# GPU call: sidecar tests, then configs 4/5 with the sidecar and without (CLONOS_SIDECAR=0)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/c45; rm -rf $O; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -m gpu -q -x --timeout 120 --timeout-method thread \
  tests/test_gpu_sidecar.py tests/test_gpu_log.py tests/test_gpu_replay.py > $O/t.log 2>&1
rc=$?; tail -2 $O/t.log; [ $rc -eq 0 ] || exit $rc
for v in side scan side scan; do
  if [ $v = scan ]; then export CLONOS_SIDECAR=0; else unset CLONOS_SIDECAR; fi
  timeout -k 10 200 python3 bench.py --config4-only > $O/$v.json 2> $O/$v.err || exit 3
  python3 - "$O/$v.json" $v <<'P'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c4, c5 = d["config4"], d["config5"]
print(sys.argv[2], "c4", c4["ms_per_step"], c4["phase_ms_rank0"], c4["kernels_rank0"]["upstream_scatter"]["avg_ms"],
      "c5", c5["latency_ms"], c5["kernels_rank0"]["upstream_scatter"]["avg_ms"])
P
done
