#!/bin/bash
# GPU call: robust resolve (speculative parallel pass), emit halo 1 KiB: robust tests + config 3.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5c8; rm -rf $O; mkdir -p $O
echo tests
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_longrec.py tests/test_gpu_decode.py tests/test_gpu_jser.py tests/test_gpu_span_fallback.py \
  tests/test_gpu_tiny.py tests/test_gpu_decode_async.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -2 $O/tests.log
echo c3
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-inflight --no-config1 --no-config4 > $O/c3.json 2> $O/c3.err || exit 3
python3 - <<'P'
import json
d=[json.loads(l) for l in open("gpurun_out/r5c8/c3.json") if l.startswith("{")][-1]
c=d["config3"]; print("fast", c["ms_per_step"], "robust", c["robust_pipeline"]["ms_per_step"], c["robust_pipeline"]["kernels_ms"])
P
echo done
