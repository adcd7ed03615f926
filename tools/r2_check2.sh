set -euo pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c2/all.log 2>&1 &&
timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-config3 --no-inflight --no-config4 > gpurun_out/c2/b.json 2>gpurun_out/c2/b.err &&
timeout -k 10 300 python3 bench.py --config4-only --no-cpu-baseline > gpurun_out/c2/c4.json 2>gpurun_out/c2/c4.err &&
echo ok
