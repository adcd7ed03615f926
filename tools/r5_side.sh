#!/bin/bash
# GPU call: the write-path sidecar -- its tests and the Serializable/decode suites, then
# config 3 with the sidecar and without (CLONOS_SIDECAR=0)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/side; rm -rf $O; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -m gpu -q -x --timeout 120 --timeout-method thread \
  tests/test_gpu_sidecar.py tests/test_gpu_jser.py tests/test_gpu_decode.py tests/test_gpu_longrec.py \
  tests/test_gpu_fused.py > $O/t.log 2>&1
rc=$?; tail -4 $O/t.log; [ $rc -eq 0 ] || exit $rc
echo c3-side && timeout -k 10 240 python3 tools/bench_config3.py > $O/c3_side.json 2> $O/c3_side.err || exit 3
echo c3-scan && CLONOS_SIDECAR=0 timeout -k 10 240 python3 tools/bench_config3.py > $O/c3_scan.json 2> $O/c3_scan.err || exit 4
python3 - <<'P'
import json
for n in ("side", "scan"):
    d = json.loads(open(f"gpurun_out/side/c3_{n}.json").read().strip().splitlines()[-1])
    print(n, {k: v for k, v in d.items() if k in ("ms_per_step", "hbm_frac", "kernels")})
P
echo prof && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p -o run --output-format csv -- python3 tools/bench_config3.py --steps 3 > $O/c3p.json 2> $O/c3p.err || exit 5
python3 - <<'P'
import csv, glob
f = glob.glob("gpurun_out/side/p/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in ("jser", "count", "emit", "scatter")):
        print(r["Name"][:48], r["Calls"], r["AverageNs"])
P
echo phases && timeout -k 10 150 python3 tools/side_phases.py 64 2>&1 | grep -v amdgpu.ids
