# A/B timing of engine builds (ab/lib<name>.so, tools/ab_build.sh) on one box, alternating,
# so that box-to-box variation does not decide.  usage: tools/ab.sh <rounds> <name>...
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"; out=gpurun_out/ab; rm -rf $out; mkdir -p $out
rounds=$1; shift
for r in $(seq 1 $rounds); do
  for v in "$@"; do
    CLONOS_LIB=$PWD/ab/lib$v.so timeout -k 10 150 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-config3 --no-inflight --no-config4 > $out/c2_${v}_$r.json 2>$out/c2_${v}_$r.err || exit 1
    [ -n "$NO_C3" ] || CLONOS_LIB=$PWD/ab/lib$v.so timeout -k 10 200 python3 tools/bench_config3.py --logs 128 --steps 3 > $out/c3_${v}_$r.json 2>$out/c3_${v}_$r.err || exit 1
  done
done
python3 - "$@" <<'PY'
import glob, json, sys
for v in sys.argv[1:]:
    c2 = [json.loads(open(f).read().strip().splitlines()[-1]) for f in sorted(glob.glob(f"gpurun_out/ab/c2_{v}_*.json"))]
    c3 = [json.loads(open(f).read().strip().splitlines()[-1]) for f in sorted(glob.glob(f"gpurun_out/ab/c3_{v}_*.json"))]
    k = lambda b, n: b["kernels_isolated"][n]["avg_ms"]
    print(v, "c2 count", [round(k(b, "decode_count"), 4) for b in c2], "emit", [round(k(b, "decode_emit"), 4) for b in c2],
          "step", [b["ms_per_step"] for b in c2],
          "| c3 count", [round(b["kernels"]["decode_count"]["avg_ms"], 3) for b in c3],
          "emit", [round(b["kernels"]["decode_emit"]["avg_ms"], 3) for b in c3],
          "jser", [round(b["kernels"].get("decode_jser", {"avg_ms": 0})["avg_ms"], 3) for b in c3],
          "step", [round(b["ms_per_step"], 3) for b in c3], "fallback", [b["kernels"].get("decode_fallback", {}).get("launches", 0) for b in c3])
PY
