#!/bin/bash
# A/B of engine settings given as environment assignments, alternating on one box:
#   tools/ab_env.sh <rounds> "<name>=<VAR=v VAR2=v2>" ...   (name=  with nothing: defaults)
# Config 2 (bench.py decode + slice leg) and config 3 (tools/bench_config3.py, 128 logs).
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"; out=gpurun_out/abenv; rm -rf $out; mkdir -p $out
rounds=$1; shift
for r in $(seq 1 $rounds); do
  for spec in "$@"; do
    name=${spec%%=*}; vars=${spec#*=}
    env $vars timeout -k 10 150 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-config3 --no-inflight --no-config4 --no-config1 > $out/c2_${name}_$r.json 2>$out/c2_${name}_$r.err || exit 1
    [ -n "$NO_C3" ] || env $vars timeout -k 10 200 python3 tools/bench_config3.py --logs 128 --steps 3 > $out/c3_${name}_$r.json 2>$out/c3_${name}_$r.err || exit 1
  done
done
names=""; for spec in "$@"; do names="$names ${spec%%=*}"; done
python3 - $names <<'PY'
import glob, json, sys
def last(f):
    return [json.loads(l) for l in open(f) if l.startswith("{")][-1]
for v in sys.argv[1:]:
    c2 = [last(f) for f in sorted(glob.glob(f"gpurun_out/abenv/c2_{v}_*.json"))]
    c3 = [last(f) for f in sorted(glob.glob(f"gpurun_out/abenv/c3_{v}_*.json"))]
    ki = lambda b, n: b["kernels_isolated"].get(n, {}).get("avg_ms")
    kt = lambda b, n: b["kernels"].get(n, {}).get("avg_ms")
    print(v, "c2 pipe", [ki(b, "decode_pipeline") for b in c2], "gather", [ki(b, "slice_gather") for b in c2],
          "gather_in_step", [kt(b, "slice_gather") for b in c2], "step", [b["ms_per_step"] for b in c2],
          "| c3 pipe", [b["kernels"].get("decode_pipeline", {}).get("avg_ms") for b in c3],
          "step", [round(b["ms_per_step"], 3) for b in c3],
          "fallback", [b["kernels"].get("decode_fallback", {}).get("launches", 0) for b in c3], flush=True)
PY
