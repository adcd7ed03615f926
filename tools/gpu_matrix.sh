#!/bin/bash
# The -m gpu suite once per developer switch that moves decodes onto another path (the sidecar
# off, the lean walk forced, kept errors off, the single-launch small path off), so that every
# path's results are held to the oracle by the whole suite.  Tests that assert which path ran
# fail under the switch that turns that path off; the logs name them.  Run under gpurun from the
# repository root: bash tools/gpu_matrix.sh [VAR=VALUE ...]  (default: the four switches)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/mx
vars=("$@")
[ ${#vars[@]} -eq 0 ] && vars=(CLONOS_SIDECAR=0 CLONOS_LEAN=1 CLONOS_KEEP_ERRORS=0 CLONOS_SMALL=0)
for v in "${vars[@]}"; do
  echo "== $v $(date +%T)"
  env "$v" timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > "gpurun_out/mx/${v%%=*}.log" 2>&1
  rc=$?
  grep -E "^FAILED|passed|failed" "gpurun_out/mx/${v%%=*}.log" | tail -12
  [ $rc -le 1 ] || exit $rc  # (1: test failures, listed above; anything else ends the call)
done
echo "== done"
