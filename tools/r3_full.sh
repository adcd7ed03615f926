# Round-end check on one MI355X (run under gpurun): the whole -m gpu suite, smoke(), then the
# profile set (tools/profile_r02.sh; summarise with tools/r02_profile_summary.py).
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/full
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full/tests.log 2>&1 || { tail -30 gpurun_out/full/tests.log; exit 1; }
tail -2 gpurun_out/full/tests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/full/smoke.log 2>&1 || { tail -20 gpurun_out/full/smoke.log; exit 1; }
tail -1 gpurun_out/full/smoke.log
bash tools/profile_r02.sh
