#!/bin/bash
# The round's GPU evidence in one call: the -m gpu suite, smoke, then tools/profile.sh (bench
# line, kernel traces, PMC passes) into gpurun_out/prof.  Summarise with
#   python tools/profile_summary.py gpurun_out/prof <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
echo tests
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/prof/gputest.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
echo smoke && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/prof/smoke.log 2>&1 &&
bash tools/profile.sh gpurun_out/prof
