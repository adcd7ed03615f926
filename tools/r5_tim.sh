#!/bin/bash
# GPU call: config 2 step with and without the kernel timing events (CLONOS_BENCH_TIMING), and a
# kernel trace for the prep kernel after the LDS-run change.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/tim; rm -rf $O; mkdir -p $O
C2="--steps 30 --warmup 3 --no-cpu-baseline --no-config3 --no-inflight --no-config4 --no-config1"
for r in 1 2; do
  for m in 1 0; do
    CLONOS_BENCH_TIMING=$m timeout -k 10 200 python3 bench.py $C2 > $O/c2_${m}_$r.json 2>$O/c2_${m}_$r.err || exit 3
    echo "timing=$m $(tail -1 $O/c2_${m}_$r.json | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-config3 --no-inflight --no-isolated --no-config4 --no-config1 > $O/trace.json 2> $O/trace.err || exit 4
python3 tools/timeline.py $O/trace 6 > $O/timeline.txt; tail -2 $O/timeline.txt
grep prep $O/timeline.txt | head -8
