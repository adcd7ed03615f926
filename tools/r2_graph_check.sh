set -euo pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/graph
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/graph/all.log 2>&1 &&
CLONOS_GRAPHS=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_decode_async.py tests/test_gpu_decode.py -x -q --timeout 200 --timeout-method thread > gpurun_out/graph/nograph.log 2>&1 &&
CLONOS_STEP_PROBE=1 timeout -k 10 200 python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-config3 --no-inflight --no-config4 > gpurun_out/graph/b.json 2>gpurun_out/graph/b.err &&
CLONOS_GRAPHS=0 CLONOS_STEP_PROBE=1 timeout -k 10 200 python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-config3 --no-inflight --no-config4 > gpurun_out/graph/b0.json 2>gpurun_out/graph/b0.err &&
echo ok
