set -euo pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prio
A="--steps 20 --warmup 3 --no-cpu-baseline --no-config3 --no-inflight --no-config4"
CLONOS_GATHER_PRIO=0 timeout -k 10 200 python3 bench.py $A > gpurun_out/prio/p0.json 2>gpurun_out/prio/p0.err &&
timeout -k 10 200 python3 bench.py $A > gpurun_out/prio/p1.json 2>gpurun_out/prio/p1.err &&
echo ok
