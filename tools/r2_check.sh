#!/bin/bash
# Round-2 GPU check: the GPU tests, then the config-4 leg alone at N=1 and as a world-2
# gloo rehearsal on the one GPU (numbers meaningless there; it exercises the N>1 path).
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/r2b}
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > "$OUT/tests.log" 2>&1 &&
timeout -k 10 300 python -u bench.py --config4-only > "$OUT/c4_n1.json" 2> "$OUT/c4_n1.err" &&
CLONOS_BENCH_REHEARSAL=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --config4-only > "$OUT/c4_n2.json" 2> "$OUT/c4_n2.err"
