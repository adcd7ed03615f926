#!/bin/bash
# GPU call: changed tests, count-pass phase profile (lean on / off), config 4/5 legs, and the
# world-4 rehearsal of bench.py --gpus 4 (every rank on GPU 0 over gloo).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5c3; rm -rf $O; mkdir -p $O
echo tests
timeout -k 10 400 python -u -m pytest tests/test_gpu_small.py tests/test_gpu_span_fallback.py tests/test_gpu_replay.py tests/test_gpu_dist.py -m gpu -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.log
[ $rc -le 1 ] || exit $rc
echo "tests lean=1"
CLONOS_LEAN=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_fused.py tests/test_gpu_longrec.py tests/test_gpu_span_fallback.py tests/test_gpu_golden.py tests/test_gpu_log.py tests/test_gpu_tiny.py -m gpu -q --timeout 120 --timeout-method thread > $O/lean_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/lean_tests.log
[ $rc -le 1 ] || exit $rc
echo ab
OUT=$O/ab bash tools/r5_ab.sh "lm0 CLONOS_LEAN=0" "lm0 CLONOS_LEAN=1" "lm1 CLONOS_LEAN=1" || exit 5
echo phases
timeout -k 10 200 python3 tools/scan_phases.py 64 > $O/phases_lean.txt 2>&1 || exit 2
CLONOS_LEAN=0 timeout -k 10 200 python3 tools/scan_phases.py 64 > $O/phases_nolean.txt 2>&1 || exit 2
echo c45
timeout -k 10 300 python3 bench.py --config4-only > $O/c45.json 2> $O/c45.err || exit 3
echo rehearsal
CLONOS_BENCH_REHEARSAL=1 timeout -k 10 600 python3 bench.py --gpus 4 --steps 5 --warmup 2 --no-cpu-baseline --config4-steps 3 --config5-steps 2 > $O/rehearsal_w4.json 2> $O/rehearsal_w4.err || exit 4
echo done
