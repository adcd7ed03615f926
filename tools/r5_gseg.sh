#!/bin/bash
# GPU call: segment-major gather -- slice/log/replay tests, then config 2 with and without it
# (CLONOS_GATHER_SEG=0/1, twice each), and the config 4/5 leg.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/gseg; rm -rf $O; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_log.py \
  tests/test_gpu_replay.py tests/test_gpu_dist.py tests/test_gpu_delta.py tests/test_gpu_config1.py > $O/t.log 2>&1 \
  || { tail -30 $O/t.log; exit 2; }
tail -2 $O/t.log
C2="--steps 20 --warmup 3 --no-cpu-baseline --no-config3 --no-inflight --no-config4 --no-config1"
for r in 1 2; do
  for m in 0 1; do
    CLONOS_GATHER_SEG=$m timeout -k 10 200 python3 bench.py $C2 > $O/c2_${m}_$r.json 2>$O/c2_${m}_$r.err || exit 3
  done
done
python3 - <<'P'
import json, glob
for f in sorted(glob.glob("gpurun_out/gseg/c2_*.json")):
    d = [json.loads(l) for l in open(f) if l.startswith("{")][-1]
    k = d["kernels"]; ki = d["kernels_isolated"]
    print(f.split("/")[-1], d["ms_per_step"], "gather", k["slice_gather"]["avg_ms"], "iso", ki["slice_gather"]["avg_ms"],
          "pipe", k["decode_pipeline"]["avg_ms"], "iso", ki["decode_pipeline"]["avg_ms"])
P
CLONOS_HOST_PROF=1 timeout -k 10 300 python3 bench.py --config4-only > $O/c45.json 2>$O/c45.err || exit 4
echo done
