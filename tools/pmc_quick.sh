set -euo pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmcq; mkdir -p $OUT
C2="--steps 2 --warmup 1 --no-cpu-baseline --no-config3 --no-inflight --no-isolated --no-config4"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $OUT/c2_sq1 -o run --output-format csv -- python3 bench.py $C2 > $OUT/c2_sq1.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_SALU SQ_BUSY_CU_CYCLES SQ_CYCLES -d $OUT/c2_sq3 -o run --output-format csv -- python3 bench.py $C2 > $OUT/c2_sq3.log 2>&1 &&
echo ok
