#!/bin/bash
# GPU call: robust-tier LDS tables + prefiltered Serializable fill, direct mapped outputs,
# 16 host threads: the decode test files, config 3's robust leg and the config 4/5 leg.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5c7; rm -rf $O; mkdir -p $O
echo tests
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_decode.py tests/test_gpu_jser.py tests/test_gpu_span_fallback.py tests/test_gpu_fused.py \
  tests/test_gpu_small.py tests/test_gpu_decode_async.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -2 $O/tests.log
echo c3
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-inflight --no-config1 --no-config4 > $O/c3.json 2> $O/c3.err || exit 3
echo c45
CLONOS_HOST_PROF=1 timeout -k 10 300 python3 bench.py --config4-only > $O/c45.json 2> $O/c45.err || exit 3
echo done
