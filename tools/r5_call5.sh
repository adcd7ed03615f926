#!/bin/bash
# GPU call: the whole -m gpu suite, smoke, the driver's default bench line, and a warm-up /
# grid-margin A/B of the count pass.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5c5; rm -rf $O; mkdir -p $O
echo tests
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/gputest.log
[ $rc -le 1 ] || exit $rc
echo smoke && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
echo bench && timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 3
echo ab
mkdir -p ab && cp clonos_amd/libclonos_engine.so ab/libcur.so
OUT=$O/ab bash tools/r5_ab.sh "cur" "cur CLONOS_WARM=64" "cur CLONOS_WARM=80" "cur CLONOS_WARM=112" "cur CLONOS_COUNT_MARGIN=0" || exit 5
echo done
