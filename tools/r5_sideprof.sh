#!/bin/bash
# GPU call: kernel trace of config 3 with the sidecar (k_decode_jser vs the general walker)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/sideprof; rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p -o run --output-format csv -- python3 tools/bench_config3.py --steps 3 > $O/c3.json 2> $O/c3.err || exit 3
f=$(find $O/p -name 'run_kernel_stats.csv' | head -1); cp "$f" $O/stats.csv
python3 - <<'P'
import csv
for r in csv.DictReader(open("gpurun_out/sideprof/stats.csv")):
    if "jser" in r["Name"] or "count" in r["Name"] or "emit" in r["Name"] or "scatter" in r["Name"]:
        print(r["Name"][:60], r["Calls"], r["AverageNs"])
P
