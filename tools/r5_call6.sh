#!/bin/bash
# GPU call: config 4/5 phase parts (host stage timers; 8 and 16 host threads), a kernel +
# memory-copy trace of that leg, and the config-3 count pass's phase profile.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5c6; rm -rf $O; mkdir -p $O
echo c45
CLONOS_HOST_PROF=1 timeout -k 10 300 python3 bench.py --config4-only > $O/c45_prof.json 2> $O/c45_prof.err || exit 3
CLONOS_HOST_THREADS=16 timeout -k 10 300 python3 bench.py --config4-only > $O/c45_t16.json 2> $O/c45_t16.err || exit 3
echo trace
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/c4_trace -o run --output-format csv -- python3 bench.py --config4-only > $O/c4_trace.log 2>&1 || exit 4
echo phases
timeout -k 10 300 python3 tools/scan_phases.py 64 c3 > $O/phases_c3.txt 2>&1 || exit 2
echo done
