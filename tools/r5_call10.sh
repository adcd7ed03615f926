#!/bin/bash
# GPU call: robust emit with select decode + lengths from phase A; robust tests; robust kernel
# times per A/B build (ab/lib*.so: jser fill stage-only / no parse, emit without phase B).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5c10; rm -rf $O; mkdir -p $O
echo tests
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_longrec.py tests/test_gpu_decode.py tests/test_gpu_jser.py tests/test_gpu_span_fallback.py \
  tests/test_gpu_tiny.py tests/test_gpu_decode_async.py tests/test_gpu_golden.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -2 $O/tests.log
for v in base j1 j2 e1; do
  echo $v
  CLONOS_NOCHECK=1 CLONOS_LIB=$PWD/ab/lib$v.so timeout -k 10 120 python3 tools/robust_run.py 64 3 2>&1 | grep robust || exit 3
done
echo done
