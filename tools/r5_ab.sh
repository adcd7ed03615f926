#!/bin/bash
# Count-pass A/B on one box: builds ab/lib<name>.so (tools/ab_build.sh) x env settings, config-2
# isolated kernel times (bench.py) and the config-3 subset (tools/bench_config3.py).
# usage: tools/r5_ab.sh "<name> <ENV=V ...>" ...   (each arg: a build name and env settings)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/r5ab}; rm -rf $OUT; mkdir -p $OUT
C2="--steps 10 --warmup 2 --no-cpu-baseline --no-config3 --no-inflight --no-config4 --no-config1"
i=0
specs=("$@")
for round in 1 2; do
  for spec in "${specs[@]}"; do
    set -- $spec; name=$1; shift
    i=$((i+1))
    env CLONOS_LIB=$PWD/ab/lib$name.so "$@" timeout -k 10 150 python3 bench.py $C2 > $OUT/c2_${i}.json 2> $OUT/c2_${i}.err || exit 1
    echo "$spec" > $OUT/c2_${i}.spec
    if [ -n "$C3" ]; then
      env CLONOS_LIB=$PWD/ab/lib$name.so "$@" timeout -k 10 200 python3 tools/bench_config3.py --logs 128 --steps 3 > $OUT/c3_${i}.json 2> $OUT/c3_${i}.err || exit 1
    fi
  done
done
python3 - <<'PY'
import glob, json, os
out = os.environ.get("OUT", "gpurun_out/r5ab")
rows = {}
for f in sorted(glob.glob(f"{out}/c2_*.json")):
    i = f.split("_")[-1].split(".")[0]
    spec = open(f"{out}/c2_{i}.spec").read().strip()
    b = json.loads(open(f).read().strip().splitlines()[-1])
    k = b["kernels_isolated"]
    r = rows.setdefault(spec, [])
    c3 = None
    if os.path.exists(f"{out}/c3_{i}.json"):
        c = json.loads(open(f"{out}/c3_{i}.json").read().strip().splitlines()[-1])
        c3 = (round(c["kernels"]["decode_count"]["avg_ms"], 4), round(c["ms_per_step"], 3))
    r.append((round(k["decode_count"]["avg_ms"], 4), round(k["decode_emit"]["avg_ms"], 4),
              round(k["decode_pipeline"]["avg_ms"], 4), b["ms_per_step"], c3))
for spec, r in rows.items():
    print(f"{spec:40s} count/emit/pipe/step(c3 count, step):", r)
PY
