#!/bin/bash
# GPU call: tests touched by the scan change, config 4/5 with host stage timers, row-pad A/B of
# the count pass with its LDS counters, and the world-4 rehearsal of bench.py --gpus 4.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5c4; rm -rf $O; mkdir -p $O
echo tests
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode_async.py tests/test_gpu_fused.py tests/test_gpu_config1.py tests/test_gpu_log.py tests/test_gpu_replay.py tests/test_gpu_dist.py -m gpu -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.log
[ $rc -le 1 ] || exit $rc
echo c45
CLONOS_HOST_PROF=1 timeout -k 10 300 python3 bench.py --config4-only > $O/c45_prof.json 2> $O/c45_prof.err || exit 3
timeout -k 10 300 python3 bench.py --config4-only > $O/c45.json 2> $O/c45.err || exit 3
echo ab
C3=1 OUT=$O/ab bash tools/r5_ab.sh "z0" "z3" || exit 5
echo pmc
C2="--steps 2 --warmup 1 --no-cpu-baseline --no-config3 --no-inflight --no-isolated --no-config4 --no-config1"
for v in z0 z3; do
  CLONOS_LIB=$PWD/ab/lib$v.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAVES -d $O/pmc_$v -o run --output-format csv -- python3 bench.py $C2 > $O/pmc_$v.log 2>&1 || exit 6
done
echo rehearsal
CLONOS_BENCH_REHEARSAL=1 timeout -k 10 600 python3 bench.py --gpus 4 --steps 5 --warmup 2 --no-cpu-baseline --config4-steps 3 --config5-steps 2 > $O/rehearsal_w4.json 2> $O/rehearsal_w4.err || exit 4
echo done
