# Warm-up sweep (CLONOS_WARM) on one MI355X: config-2 count and config-3 (128-log subset) count.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"; out=gpurun_out/warm; rm -rf $out; mkdir -p $out
for w in 96 128 160 192; do
  CLONOS_WARM=$w timeout -k 10 150 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-config3 --no-inflight --no-config4 > $out/c2_$w.json 2>/dev/null || exit 1
done
for w in; do
  CLONOS_WARM=$w timeout -k 10 200 python3 tools/bench_config3.py --logs 128 --steps 3 > $out/c3_$w.json 2>/dev/null || exit 1
done
python3 - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/warm/*.json")):
    b = json.loads(open(f).read().strip().splitlines()[-1])
    k = b.get("kernels_isolated", b.get("kernels"))
    print(f.split("/")[-1], "count", round(k["decode_count"]["avg_ms"], 4), "step", b["ms_per_step"])
PY
