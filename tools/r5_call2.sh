#!/bin/bash
# GPU call: the decode tests with the lean walk forced on every batch, then the count A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5c2
echo "tests lean=1"
CLONOS_LEAN=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_fused.py tests/test_gpu_longrec.py tests/test_gpu_span_fallback.py tests/test_gpu_golden.py tests/test_gpu_log.py tests/test_gpu_decode_async.py tests/test_gpu_tiny.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r5c2/lean_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r5c2/lean_tests.log
[ $rc -le 1 ] || exit $rc
echo ab
C3=1 OUT=gpurun_out/r5c2/ab bash tools/r5_ab.sh "s1 CLONOS_LEAN=0" "s1 CLONOS_LEAN=1" "s3 CLONOS_LEAN=1" "s3 CLONOS_LEAN=1 CLONOS_WARM=64" "s3 CLONOS_LEAN=1 CLONOS_WARM=80" || exit 5
echo pmc
C2="--steps 2 --warmup 1 --no-cpu-baseline --no-config3 --no-inflight --no-isolated --no-config4 --no-config1"
for v in 0 1; do
  CLONOS_LEAN=$v timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d gpurun_out/r5c2/pmc1_$v -o run --output-format csv -- python3 bench.py $C2 > gpurun_out/r5c2/pmc1_$v.log 2>&1 || exit 6
  CLONOS_LEAN=$v timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE -d gpurun_out/r5c2/pmc2_$v -o run --output-format csv -- python3 bench.py $C2 > gpurun_out/r5c2/pmc2_$v.log 2>&1 || exit 6
done
echo done
