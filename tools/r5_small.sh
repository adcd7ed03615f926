#!/bin/bash
# GPU call: the small-decode group (empty batches, per-tile launch, config 1/5 paths)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/small; rm -rf $O; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -m gpu -q --timeout 120 --timeout-method thread \
  tests/test_gpu_decode.py tests/test_gpu_golden.py tests/test_gpu_jser.py tests/test_gpu_small.py \
  tests/test_gpu_config1.py tests/test_gpu_replay.py tests/test_gpu_tiny.py tests/test_gpu_decode_async.py > $O/t.log 2>&1
rc=$?; tail -5 $O/t.log; exit $rc
