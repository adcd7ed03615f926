#!/bin/bash
# One GPU call: the -m gpu suite (or the test files given as arguments), then the default bench
# line and an A/B-style config-2/3 kernel line per engine build in ab/ (if any).  Output under
# gpurun_out/suite.  usage (under gpurun): bash tools/gpu_suite.sh [test files...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/suite; mkdir -p $out
tests=${*:-tests}
echo "tests: $tests"
timeout -k 10 1500 python -u -m pytest $tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $out/pytest.log
[ $rc -le 1 ] || exit $rc
echo bench && timeout -k 10 400 python3 bench.py > $out/bench.json 2> $out/bench.err
echo "bench rc=$?"
