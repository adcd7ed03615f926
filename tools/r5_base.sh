#!/bin/bash
# Round-5 baseline: config-2 bench with host split, plus a kernel trace for tools/timeline.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5base; mkdir -p $OUT
C2="--steps 20 --warmup 3 --no-cpu-baseline --no-config3 --no-inflight --no-config4 --no-config1"
echo b1 && CLONOS_STEP_PROBE=1 timeout -k 10 200 python3 bench.py $C2 > $OUT/b1.json 2> $OUT/b1.err &&
echo b2 && CLONOS_HOST_PROF=1 timeout -k 10 200 python3 bench.py $C2 > $OUT/b2.json 2> $OUT/b2.err &&
echo trace && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-config3 --no-inflight --no-isolated --no-config4 --no-config1 > $OUT/trace.log 2>&1 &&
python3 tools/timeline.py $OUT/trace 3 > $OUT/timeline.txt && echo done
