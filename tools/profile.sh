#!/bin/bash
# Profile of the bench on one MI355X (run under gpurun from the repo root; summarise with
# tools/profile_summary.py <dir> <tag>).
#   bench.json                full bench line (config 2 + config 3 + in-flight + config 4, CPU baselines)
#   trace/                    rocprofv3 --kernel-trace --stats over the config-2 bench (the roofline kernel)
#   c2_fetch, c2_write        FETCH_SIZE / WRITE_SIZE passes, config 2
#   c2_sq1..c2_sq3            SQ counter groups (instructions, waits, LDS, VALU lane cycles), config 2
#   c3_trace, c3_fetch, c3_write, c3_sq1..c3_sq3   the same for config 3 (tools/bench_config3.py)
#   ifl_trace                 rocprofv3 --stats over the in-flight replay leg alone
#   c4_trace                  rocprofv3 --stats over the config-4 / config-5 legs alone
# Counters only ever with --kernel-trace (no sys/runtime trace); one group per pass, each
# within the per-block limits; every GPU step has its own time limit; steps chained with &&.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/prof}
mkdir -p "$OUT"
C2="--steps 2 --warmup 1 --no-cpu-baseline --no-config3 --no-inflight --no-isolated --no-config4 --no-config1"
C3="--logs 256 --steps 1"
SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
SQ2="SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
SQ3="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_SALU SQ_BUSY_CU_CYCLES SQ_CYCLES"
pmc() {  # pmc <dir> <counters> <program...>
  local d=$1 c=$2; shift 2
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $c -d "$OUT/$d" -o run --output-format csv -- "$@" > "$OUT/$d.log" 2>&1
}
echo "bench" && timeout -k 10 600 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" &&
echo "trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-config3 --no-inflight --no-isolated --no-config4 --no-config1 > "$OUT/trace.log" 2>&1 &&
echo "c2 pmc" && pmc c2_fetch FETCH_SIZE python3 bench.py $C2 && pmc c2_write WRITE_SIZE python3 bench.py $C2 &&
pmc c2_sq1 "$SQ1" python3 bench.py $C2 && pmc c2_sq2 "$SQ2" python3 bench.py $C2 && pmc c2_sq3 "$SQ3" python3 bench.py $C2 &&
echo "c3" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/c3_trace" -o run --output-format csv -- \
    python3 tools/bench_config3.py --logs 256 --steps 3 > "$OUT/c3_trace.log" 2>&1 &&
pmc c3_fetch FETCH_SIZE python3 tools/bench_config3.py $C3 && pmc c3_write WRITE_SIZE python3 tools/bench_config3.py $C3 &&
pmc c3_sq1 "$SQ1" python3 tools/bench_config3.py $C3 && pmc c3_sq2 "$SQ2" python3 tools/bench_config3.py $C3 &&
pmc c3_sq3 "$SQ3" python3 tools/bench_config3.py $C3 &&
echo "ifl" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/ifl_trace" -o run --output-format csv -- \
    python3 bench.py --inflight-only --no-cpu-baseline > "$OUT/ifl_trace.log" 2>&1 &&
echo "c4" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/c4_trace" -o run --output-format csv -- \
    python3 bench.py --config4-only > "$OUT/c4_trace.log" 2>&1 &&
echo "done"
