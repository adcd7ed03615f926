cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/warm2
for w in 96 128 160 192 256; do
  CLONOS_WARM=$w timeout -k 10 150 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-config3 --no-inflight --no-config4 > gpurun_out/warm2/w$w.json 2>/dev/null || break
done
CLONOS_WARM=160 timeout -k 10 200 python3 tools/bench_config3.py --logs 128 --steps 3 > gpurun_out/warm2/c3_160.json 2>/dev/null
CLONOS_WARM=96 timeout -k 10 200 python3 tools/bench_config3.py --logs 128 --steps 3 > gpurun_out/warm2/c3_96.json 2>/dev/null
echo done
