#!/bin/bash
# GPU call: robust-pipeline tests with the sidecar, then config 3 forced robust with and without it
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/rob2; rm -rf $O; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -m gpu -q -x --timeout 120 --timeout-method thread \
  tests/test_gpu_sidecar.py tests/test_gpu_jser.py tests/test_gpu_span_fallback.py tests/test_gpu_longrec.py tests/test_gpu_fused.py > $O/t.log 2>&1
rc=$?; tail -2 $O/t.log; [ $rc -eq 0 ] || exit $rc
for v in side scan; do
  if [ $v = scan ]; then export CLONOS_SIDECAR=0; else unset CLONOS_SIDECAR; fi
  timeout -k 10 300 python3 tools/bench_config3.py --decode robust --steps 3 > $O/$v.json 2> $O/$v.err || exit 3
  python3 - "$O/$v.json" $v <<'P'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d.get("ms_per_step"), {k: v.get("avg_ms") for k, v in d.get("kernels", {}).items()})
P
done
