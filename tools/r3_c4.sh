#!/bin/bash
# Config 4 at N=1 with two engine builds (ab/libtiny0.so: no lane-per-span count path,
# ab/libtiny1.so: with it), then a kernel trace of the second.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r3c4; mkdir -p $OUT
for v in tiny0 tiny1 tiny0 tiny1; do
  CLONOS_LIB=$PWD/ab/lib$v.so timeout -k 10 200 python3 -u bench.py --config4-only > $OUT/c4_$v.json 2> $OUT/c4_$v.err || exit 1
  python3 -c "import json,sys; d=[json.loads(l) for l in open('$OUT/c4_$v.json') if l.startswith('{')][-1]['config4']; print('$v', d['ms_per_step'], d['phase_ms_rank0'], {k: v['avg_ms'] for k, v in d['kernels_rank0'].items()})"
done
CLONOS_LIB=$PWD/ab/libtiny1.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --config4-only > $OUT/trace.log 2>&1
