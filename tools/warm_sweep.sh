# Sweep the speculative warm-up (CLONOS_WARM) on config 2 and a config-3 subset.
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT; out=gpurun_out/${1:-warm}; mkdir -p $out
for w in ${WARMS:-0 16 32 48 64 96}; do
  CLONOS_WARM=$w timeout -k 10 150 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-config3 --no-inflight --no-config4 > $out/w$w.json 2>$out/w$w.err || exit 1
  CLONOS_WARM=$w timeout -k 10 200 python3 tools/bench_config3.py --logs 128 --steps 3 > $out/c3_$w.json 2>$out/c3_$w.err || exit 1
done
echo done
