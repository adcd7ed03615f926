#!/bin/bash
# GPU call: robust tier (next-tile tables, resolve far walk from tables): tests, config 3, and
# counters of the robust kernels (tools/robust_run.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5c9; rm -rf $O; mkdir -p $O
echo tests
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_longrec.py tests/test_gpu_decode.py tests/test_gpu_jser.py tests/test_gpu_span_fallback.py \
  tests/test_gpu_tiny.py tests/test_gpu_decode_async.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -2 $O/tests.log
echo run
timeout -k 10 120 python3 tools/robust_run.py 64 3 > $O/run.log 2>&1 || { tail $O/run.log; exit 3; }
cat $O/run.log
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
           "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp -d $O/p$i -o run --output-format csv -- python3 tools/robust_run.py 64 2 > $O/p$i.log 2>&1 || exit 4
done
python3 tools/pmc_summary.py $O > $O/pmc.txt
echo c3
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-inflight --no-config1 --no-config4 > $O/c3.json 2> $O/c3.err || exit 3
python3 - <<'P'
import json
d=[json.loads(l) for l in open("gpurun_out/r5c9/c3.json") if l.startswith("{")][-1]
c=d["config3"]; print("fast", c["ms_per_step"], "robust", c["robust_pipeline"]["ms_per_step"], c["robust_pipeline"]["kernels_ms"])
P
echo done
