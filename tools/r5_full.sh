#!/bin/bash
# GPU call: the whole -m gpu suite, smoke, and the default bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/full; rm -rf $O; mkdir -p $O
echo suite
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; tail -3 $O/gputest.log; [ $rc -eq 0 ] || exit $rc
echo smoke && timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
echo bench && timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 4
python3 - <<'P'
import json
d=[json.loads(l) for l in open("gpurun_out/full/bench.json") if l.startswith("{")][-1]
print("value", d["value"], "ms", d["ms_per_step"], "roof", d["roofline"]["frac"], "cpu", d["cpu_baseline"]["value"])
print("c3", d["config3"]["ms_per_step"], d["config3"].get("ms_per_step_one_at_a_time"), d["config3"]["hbm_frac"], "robust", d["config3"]["robust_pipeline"]["ms_per_step"])
print("c4", d["config4"]["ms_per_step"], "c5", d["config5"]["latency_ms"], d["config5"]["phase_ms_max_over_ranks"])
print("c1", {k: v for k, v in d["config1"].items() if "ms" in k})
P
