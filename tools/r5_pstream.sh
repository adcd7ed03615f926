#!/bin/bash
# GPU call: plan upload on a side stream -- async/decode tests, config 2 A/B (CLONOS_PLAN_STREAM),
# and a kernel trace for the decode-to-decode gap.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pst; rm -rf $O; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_decode_async.py \
  tests/test_gpu_fused.py tests/test_gpu_log.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 2; }
tail -1 $O/t.log
C2="--steps 30 --warmup 3 --no-cpu-baseline --no-config3 --no-inflight --no-config4 --no-config1"
for r in 1 2; do
  for m in 0 1; do
    CLONOS_PLAN_STREAM=$m timeout -k 10 200 python3 bench.py $C2 > $O/c2_${m}_$r.json 2>$O/c2_${m}_$r.err || exit 3
    echo "plan_stream=$m $(tail -1 $O/c2_${m}_$r.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernels"]["decode_pipeline"]["avg_ms"])')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-config3 --no-inflight --no-isolated --no-config4 --no-config1 > $O/trace.json 2> $O/trace.err || exit 4
python3 tools/timeline.py $O/trace 8 --summary
