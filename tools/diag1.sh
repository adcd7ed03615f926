set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/diag1
timeout -k 10 120 python3 tools/scan_phases.py 16 > gpurun_out/diag1/phases_c2.txt 2>&1 &&
timeout -k 10 120 python3 tools/scan_phases.py 16 c3 > gpurun_out/diag1/phases_c3.txt 2>&1 &&
bash tools/pmc.sh gpurun_out/diag1/pmc_c2 --logs 16 --steps 2 --warmup 1 --no-cpu-baseline --no-config3 --no-inflight --no-isolated &&
bash tools/pmc_c3.sh
