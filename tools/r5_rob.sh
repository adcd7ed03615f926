#!/bin/bash
# GPU call: robust tier probe (phase stamps), robust tests, config-3 bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python3 tools/robust_phases.py 64 || exit 1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_longrec.py \
  tests/test_gpu_jser.py tests/test_gpu_span_fallback.py tests/test_gpu_decode.py tests/test_gpu_tiny.py > gpurun_out/t.log 2>&1 \
  || { tail -30 gpurun_out/t.log; exit 2; }
tail -2 gpurun_out/t.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-inflight --no-config1 --no-config4 > gpurun_out/c3.json 2>gpurun_out/c3.err || exit 3
python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/c3.json') if l.startswith('{')][-1]
c=d['config3']; print('fast', c['ms_per_step'], 'robust', c['robust_pipeline']['ms_per_step'], c['robust_pipeline']['kernels_ms'])"
