set -euo pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/dc
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_decode.py tests/test_gpu_decode_async.py tests/test_gpu_golden.py tests/test_gpu_replay.py -x -q --timeout 100 --timeout-method thread > gpurun_out/dc/t.log 2>&1 &&
timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-config3 --no-inflight --no-config4 > gpurun_out/dc/b.json 2>gpurun_out/dc/b.err &&
timeout -k 10 200 python3 tools/bench_config3.py --logs 256 --steps 3 > gpurun_out/dc/c3.json 2>gpurun_out/dc/c3.err &&
echo ok
