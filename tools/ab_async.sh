set -euo pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/async
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode_async.py -x -q --timeout 200 --timeout-method thread > gpurun_out/async/t1.log 2>&1 &&
A="--steps 20 --warmup 3 --no-cpu-baseline --no-config3 --no-inflight --no-config4"
CLONOS_GATHER_PRIO=0 timeout -k 10 200 python3 bench.py $A > gpurun_out/async/p0.json 2>gpurun_out/async/p0.err &&
timeout -k 10 200 python3 bench.py $A > gpurun_out/async/p1.json 2>gpurun_out/async/p1.err &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/async/all.log 2>&1 &&
echo ok
